/*
 * oracle.h -- TEST INFRASTRUCTURE. CPU restatement of the reference PMVS patch
 * loop (manlito/densepoints methods/pmvs + modules/core).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this; the
 * product (densepoints_amd/) never links it.
 *
 * Parity status: PINNED for NCCScore (tests/core/test_error_functions.cpp:9-15)
 * and View decomposition (tests/core/test_projection_matrix_decomposition.cpp:
 * 13-35); every OpenCV-internal step (findHomography, warpPerspective fixed
 * point, BGR2GRAY, DownhillSolver) is restated from OpenCV 3.4 semantics and
 * is "parity unpinned" against the reference binary, which cannot be built
 * here (needs OpenCV+contrib, PCL, Eigen, GTest).
 *
 * Record layouts below are byte-identical to include/densepoints.h on purpose
 * (tests hand the same numpy buffers to both); they are declared separately
 * so the oracle shares no source with the product.
 */
#ifndef DP_ORACLE_H
#define DP_ORACLE_H

#include <stdint.h>

#define OR_MAX_VIEWS 128
#define OR_MAX_CELL 32

typedef struct or_options {
    int32_t seed_cell_size;       /* 16  matcher.h:25 (Seed uses MatcherOptions::cell_size) */
    int32_t expand_cell_size;     /* 11  expand.h:12 */
    int32_t grid_scale;           /* 8   patch_organizer.h:43 */
    int32_t max_patches_per_cell; /* 1   patch_organizer.h:42 */
    int32_t min_visible;          /* 3   optimization.h:17 */
    int32_t min_expand_visible;   /* 2   expand.cpp:67 */
    int32_t nm_max_evals;         /* 500 optimization_opencv.cpp:60 */
    int32_t reserved0;
    double ncc_threshold;         /* 0.6  optimization.h:16 */
    double visible_angle;         /* 0.78 patch.h:56 */
    double candidate_angle;       /* 1.04 patch.h:57 */
    double nm_step[3];            /* 0.02,0.2,0.2 optimization_opencv.cpp:56 */
    double nm_eps;                /* 1e-4 optimization_opencv.cpp:60 */
    double ncc_denom_min;         /* 0.1  error_measurements.cpp:57 */
    int64_t max_pops;             /* 1e7  expand.cpp:95 */
} or_options;

typedef struct or_patch {
    float pos[3];
    float normal[3];
    uint32_t ref;
    uint32_t seq;      /* organizer index (queue index) */
    uint64_t vis[2];   /* visible_images_ as bitmask (lists are ascending) */
    uint64_t cand[2];  /* candidate_images_ */
    float score;       /* mean NCC of the last filter evaluation (extension) */
    uint32_t evals;    /* objective evaluations spent (E) */
    uint8_t rgb[3];
    uint8_t flags;     /* bit0 accepted, bit1 degenerate (dx==0) */
    uint32_t parent;   /* parent queue index, 0xFFFFFFFF for seeds */
} or_patch;

#define OR_FLAG_ACCEPTED 1u
#define OR_FLAG_DEGENERATE 2u

typedef struct or_scene or_scene;

/* refine modes: which reference call sequence to apply per patch */
#define OR_MODE_EVAL 0        /* scores only (no mutation)                           */
#define OR_MODE_FILTER 1      /* Optimization::FilterByErrorMeasurement             */
#define OR_MODE_NM 2          /* OptimizationOpenCV::Optimize                        */
#define OR_MODE_SEED 3        /* Seed::FilterPatches then OptimizePatches (seed.cpp) */
#define OR_MODE_EXPAND 4      /* Optimize -> InitRelatedImages -> Filter (expand.cpp)*/
#define OR_MODE_FAST_EVAL 5   /* performance mode: one evaluation (or_fast.c)        */
#define OR_MODE_FAST_REFINE 6 /* performance mode: CG -> InitRelatedImages -> filter */

/* performance-mode options (layout of include/densepoints.h dp_fast_options) */
typedef struct or_fast_options {
    int32_t iters;        /* conjugate-gradient iterations                   */
    int32_t margin;       /* tile margin around the initial window, pixels   */
    int32_t tile_budget;  /* bytes of gray tiles per patch                   */
    int32_t max_views;    /* staged views per patch (<= 32)                  */
    float fd_step;        /* forward-difference step, scaled units           */
    float ls_step;        /* initial line-search step, scaled units          */
    int32_t densify;      /* product only: fast expansions in dp_densify     */
    int32_t gradient;     /* 0: forward differences (spec v3), 1: analytic gradient (v4) */
    int32_t filter_max_views; /* staged views of the scoring stagings (filter, FAST_EVAL); 0 = max_views (v5) */
} or_fast_options;

#ifdef __cplusplus
extern "C" {
#endif

void or_default_options(or_options *o);
int or_view_geometry(const double P[12], double C[3], double K[9], double E[12], double xaxis[3]);
double or_ncc_int(const int32_t *a, const int32_t *b, int n, double denom_min);
void or_sincos(double x, double *s, double *c);
double or_acos(double x);

or_scene *or_scene_create(int V, const double *P, const int32_t *W, const int32_t *H,
                          const uint8_t *const *bgr, const or_options *opt);
void or_scene_destroy(or_scene *s);
int or_scene_view_info(const or_scene *s, int v, double C[3], double xr[3]);

int or_texture(const or_scene *s, int view, const double corners[12], int cell, int32_t *gray);
int or_init_related(const or_scene *s, or_patch *p);
int or_scores(const or_scene *s, const or_patch *p, const double nn[3], const double pp[3],
              int cell, double *scores, int *degenerate);
double or_objective(const or_scene *s, const or_patch *p, const double x[3], int cell);
int or_refine_batch(const or_scene *s, or_patch *p, int n, int cell, int mode,
                    uint8_t *accept, int nthreads);
int or_seeds_to_patches(const or_scene *s, const double *xyz, int n, or_patch *out);
int or_expand_children(const or_scene *s, const or_patch *parent, or_patch out[4], uint8_t acc[4]);
int or_expand_batch(const or_scene *s, const or_patch *parents, int n, or_patch *children,
                    uint8_t *acc, int nthreads);
int64_t or_densify(const or_scene *s, const double *seeds, int nseeds, or_patch *out,
                   int64_t cap, int64_t *n_seed_patches, int64_t *pops);
/* organizer object (generation-at-a-time densify tests) */
typedef struct or_org or_org;
or_org *or_org_create(const or_scene *s);
void or_org_destroy(or_org *o);
int or_org_insert(or_org *o, const or_patch *p, uint32_t seq, uint32_t parent, or_patch *out);
void or_color(const or_scene *s, or_patch *p);
/* cv::pyrDown (OpenCV 3.4 imgproc/pyramids.cpp pyrDown_: 5x5 kernel
 * [1 4 6 4 1]^T[1 4 6 4 1]/256, BORDER_REFLECT_101, dst ((W+1)/2, (H+1)/2),
 * CV_DESCALE(sum, 8)) on a BGR8 image; out holds dw*dh*3 bytes. */
int or_pyr_down(const uint8_t *bgr, int W, int H, uint8_t *out);
/* PMVS-style filter (the spec of include/densepoints.h dp_filter_patches; no
 * reference implementation exists: pmvs.h:27 is undefined, modules/filtering
 * is empty).  passes: bit 0 visibility consistency, bit 1 neighbourhood. */
#define OR_FILTER_VISIBILITY 1
#define OR_FILTER_NEIGHBORS 2
int or_filter_patches(const or_scene *s, const or_patch *p, int64_t n, int passes, double min_neighbor_frac,
                      uint8_t *keep);

/* performance mode (or_fast.c) */
void or_fast_default_options(or_fast_options *f);
int or_gray_plane(const or_scene *s, int view, uint8_t *out);
/* ROI trace (tools/roi_footprint.py; single-threaded): 5 int32 per record */
void or_trace_set(int32_t *buf, int64_t cap_records);
int64_t or_trace_count(void);
/* spec v4 gradient quantiser: rint(dncc 2^24) saturated to int32 (NaN -> INT32_MIN) */
int32_t or_fast_grad_q24(double dncc);
int or_fast_grad_probe(const or_scene *s, const or_patch *p, int cell, const or_fast_options *fo, int32_t *f,
                       float g[3]);
int or_fast_refine_batch(const or_scene *s, or_patch *p, int n, int cell, int mode, const or_fast_options *fo,
                         uint8_t *accept, int nthreads);
int or_fast_expand_batch(const or_scene *s, const or_patch *parents, int n, const or_fast_options *fo,
                         or_patch *children, uint8_t *acc, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
