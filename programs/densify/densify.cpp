// densify -- command-line front end of the MI355X patch loop.
//
// Mirrors the reference's programs/densify/main.cpp (-i scene.json, -s
// settings.json; PMVS::AddCamera per view, then PMVS::Run) and adds what
// SURVEY 8b asks of the build: -o out.ply (PMVS::PrintCloud format), --seeds
// (seed points from a file instead of Matcher::GenerateSeeds), --device,
// option overrides.  All compute goes through the C ABI of libdensepoints.so
// (include/densepoints.h): dp_set_views, dp_generate_seeds, dp_densify.
//
//   densify -i scene.json [--seeds seeds.xyz] [-s settings.json] [-o points.ply]
//           [--device N] [--max-pops N] [--level L] [--filter] [--check-only]
//           [--features N] [--fast-threshold T] [--epipolar-matching] [--matcher knn|flann]
//           [--detector orb|akaze] [--akaze-threshold T]
//   densify --synthetic V,W,H,KIND --write-scene DIR   (deterministic test scene
//           written as scene.json + PPM images + seeds.xyz; no GPU needed)
#include "scene_io.h"

#include "../../include/densepoints.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <algorithm>
#include <sys/stat.h>
#include <thread>
#include <vector>

namespace {

void usage()
{
    std::fprintf(stderr,
                 "usage: densify -i scene.json [--seeds seeds.xyz] [-s settings.json] [-o points.ply]\n"
                 "               [--device N] [--max-pops N] [--level L] [--filter] [--check-only]\n"
                 "               [--features N] [--fast-threshold T] [--epipolar-matching]\n"
                 "               [--matcher knn|flann]  (MatcherType, matcher.h:12)\n"
                 "               [--detector orb|akaze] [--akaze-threshold T]  (DetectorType, matcher.h:11)\n"
                 "               [--gpus N]   (one context per GPU, generations partitioned by\n"
                 "                             reference-view super-tile, accepted candidates\n"
                 "                             all-gathered device to device; output identical to 1 GPU)\n"
                 "               [--exchange auto|rccl|copy]  (auto: RCCL when every context has its\n"
                 "                             own GPU, else peer copies; --multi: that protocol at 1 GPU)\n"
                 "               [--replicate-below N]  (generations of fewer items run on every\n"
                 "                             context, device-resident, no exchange; default 1024 x gpus)\n"
                 "               [--mode parity|fast] [--fast-iters N] [--fast-gradient 0|1]\n"
                 "                            (fast: the performance-mode refine -- LDS-staged gray\n"
                 "                             tiles, fused CG -- for the seed stage and every expansion;\n"
                 "                             gradient 1: analytic, 0: forward differences)\n"
                 "       densify --synthetic V,W,H,KIND --write-scene DIR\n");
}

// settings JSON: any dp_options field by name (reference defaults otherwise)
void apply_settings(const dpio::Json &j, dp_options &o)
{
    if (j.kind != dpio::Json::Object)
        throw std::runtime_error("settings: expected a JSON object");
    for (const auto &kv : j.obj) {
        const std::string &k = kv.first;
        const double v = kv.second.num;
        if (k == "seed_cell_size") o.seed_cell_size = (int32_t)v;
        else if (k == "expand_cell_size") o.expand_cell_size = (int32_t)v;
        else if (k == "grid_scale") o.grid_scale = (int32_t)v;
        else if (k == "max_patches_per_cell") o.max_patches_per_cell = (int32_t)v;
        else if (k == "min_visible") o.min_visible = (int32_t)v;
        else if (k == "min_expand_visible") o.min_expand_visible = (int32_t)v;
        else if (k == "nm_max_evals") o.nm_max_evals = (int32_t)v;
        else if (k == "ncc_threshold") o.ncc_threshold = v;
        else if (k == "visible_angle") o.visible_angle = v;
        else if (k == "candidate_angle") o.candidate_angle = v;
        else if (k == "nm_eps") o.nm_eps = v;
        else if (k == "ncc_denom_min") o.ncc_denom_min = v;
        else if (k == "max_pops") o.max_pops = (int64_t)v;
        else if (k == "nm_step" && kv.second.kind == dpio::Json::Array && kv.second.arr.size() == 3)
            for (int i = 0; i < 3; ++i) o.nm_step[i] = kv.second.arr[i].num;
        else
            throw std::runtime_error("settings: unknown option '" + k + "'");
    }
}

void write_ppm(const std::string &path, int w, int h, const std::vector<uint8_t> &bgr)
{
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f)
        throw std::runtime_error("cannot write " + path);
    std::fprintf(f, "P6\n%d %d\n255\n", w, h);
    std::vector<uint8_t> rgb(bgr.size());
    for (size_t i = 0; i < bgr.size(); i += 3) {
        rgb[i] = bgr[i + 2];
        rgb[i + 1] = bgr[i + 1];
        rgb[i + 2] = bgr[i];
    }
    std::fwrite(rgb.data(), 1, rgb.size(), f);
    std::fclose(f);
}

int write_synthetic(const std::string &spec, const std::string &dir)
{
    dp_synth_config cfg;
    dp_synth_default(&cfg);
    if (std::sscanf(spec.c_str(), "%d,%d,%d,%d", &cfg.n_views, &cfg.width, &cfg.height, &cfg.kind) != 4)
        throw std::runtime_error("--synthetic expects V,W,H,KIND");
    std::vector<double> P(12 * (size_t)cfg.n_views);
    if (dp_synth_cameras(&cfg, P.data()) != DP_OK)
        throw std::runtime_error("dp_synth_cameras failed");
    mkdir(dir.c_str(), 0755);
    FILE *js = std::fopen((dir + "/scene.json").c_str(), "wb");
    if (!js)
        throw std::runtime_error("cannot write " + dir + "/scene.json");
    std::fprintf(js, "{\n  \"imagesPath\": \"%s\",\n  \"views\": [\n", dir.c_str());
    for (int v = 0; v < cfg.n_views; ++v) {
        std::vector<uint8_t> bgr((size_t)cfg.width * cfg.height * 3);
        if (dp_synth_render_host(&cfg, P.data(), v, bgr.data()) != DP_OK)
            throw std::runtime_error("dp_synth_render_host failed");
        char name[64];
        std::snprintf(name, sizeof name, "view_%03d.ppm", v);
        write_ppm(dir + "/" + name, cfg.width, cfg.height, bgr);
        std::fprintf(js, "    {\"filename\": \"%s\", \"projectionMatrix\": [", name);
        for (int r = 0; r < 3; ++r)
            std::fprintf(js, "[%.17g, %.17g, %.17g, %.17g]%s", P[12 * v + 4 * r], P[12 * v + 4 * r + 1],
                         P[12 * v + 4 * r + 2], P[12 * v + 4 * r + 3], r < 2 ? ", " : "");
        std::fprintf(js, "]}%s\n", v + 1 < cfg.n_views ? "," : "");
    }
    std::fprintf(js, "  ]\n}\n");
    std::fclose(js);
    const int64_t n = dp_synth_seeds(&cfg, P.data(), nullptr, 0);
    std::vector<double> xyz(3 * (size_t)n);
    dp_synth_seeds(&cfg, P.data(), xyz.data(), n);
    FILE *sf = std::fopen((dir + "/seeds.xyz").c_str(), "wb");
    if (!sf)
        throw std::runtime_error("cannot write seeds.xyz");
    for (int64_t i = 0; i < n; ++i)
        std::fprintf(sf, "%.17g %.17g %.17g\n", xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
    std::fclose(sf);
    std::printf("{\"scene\": \"%s/scene.json\", \"views\": %d, \"seeds\": %lld}\n", dir.c_str(), cfg.n_views,
                (long long)n);
    return 0;
}

// The exchange of the device protocol between the contexts of this process:
// RCCL (ncclAllGather of the rank slots in one ncclGroup, over xGMI) when
// every context has its own device, else device-to-device peer copies (the
// contexts share a GPU, as on a one-GPU box).
struct Exchange {
    int G = 0;
    bool rccl = false;
    std::vector<int> dev;
    std::vector<hipStream_t> stream;
    std::vector<hipEvent_t> ready; // each context's slot is complete
    std::vector<ncclComm_t> comm;
    std::vector<dp_patch *> slot, recv;
    std::vector<size_t> slot_cap, recv_cap; // records
    std::string err;

    bool hip(hipError_t e, const char *what)
    {
        if (e == hipSuccess)
            return true;
        err = std::string(what) + ": " + hipGetErrorString(e);
        return false;
    }
    bool init(const std::vector<int> &devices, const char *mode)
    {
        G = (int)devices.size();
        dev = devices;
        std::vector<int> sorted(devices);
        std::sort(sorted.begin(), sorted.end());
        const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
        rccl = std::strcmp(mode, "rccl") == 0 || (std::strcmp(mode, "auto") == 0 && distinct);
        if (rccl && !distinct) {
            err = "--exchange rccl needs one device per context";
            return false;
        }
        stream.assign(G, nullptr);
        ready.assign(G, nullptr);
        slot.assign(G, nullptr);
        recv.assign(G, nullptr);
        slot_cap.assign(G, 0);
        recv_cap.assign(G, 0);
        for (int g = 0; g < G; ++g) {
            if (!hip(hipSetDevice(dev[g]), "hipSetDevice") ||
                !hip(hipStreamCreateWithFlags(&stream[g], hipStreamNonBlocking), "hipStreamCreate") ||
                !hip(hipEventCreateWithFlags(&ready[g], hipEventDisableTiming), "hipEventCreate"))
                return false;
        }
        if (rccl) {
            comm.assign(G, nullptr);
            const ncclResult_t r = ncclCommInitAll(comm.data(), G, dev.data());
            if (r != ncclSuccess) {
                err = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
                return false;
            }
        }
        return true;
    }
    // slot: stride + 1 records; recv: G slots
    bool reserve(int64_t stride)
    {
        const size_t need = (size_t)stride + 1;
        for (int g = 0; g < G; ++g) {
            if (!hip(hipSetDevice(dev[g]), "hipSetDevice"))
                return false;
            if (slot_cap[g] < need) {
                if (slot[g] && !hip(hipFree(slot[g]), "hipFree"))
                    return false;
                slot_cap[g] = need + need / 4;
                if (!hip(hipMalloc(&slot[g], slot_cap[g] * sizeof(dp_patch)), "hipMalloc"))
                    return false;
            }
            if (recv_cap[g] < need * G) {
                if (recv[g] && !hip(hipFree(recv[g]), "hipFree"))
                    return false;
                recv_cap[g] = (need + need / 4) * G;
                if (!hip(hipMalloc(&recv[g], recv_cap[g] * sizeof(dp_patch)), "hipMalloc"))
                    return false;
            }
        }
        return true;
    }
    // every context's slot into every context's recv, rank order (queued on
    // the contexts' streams after their compaction: no host wait)
    bool all_gather(int64_t stride)
    {
        const size_t bytes = ((size_t)stride + 1) * sizeof(dp_patch);
        if (rccl) {
            ncclGroupStart();
            for (int g = 0; g < G; ++g) {
                const ncclResult_t r = ncclAllGather(slot[g], recv[g], bytes, ncclUint8, comm[g], stream[g]);
                if (r != ncclSuccess) {
                    ncclGroupEnd();
                    err = std::string("ncclAllGather: ") + ncclGetErrorString(r);
                    return false;
                }
            }
            const ncclResult_t r = ncclGroupEnd();
            if (r != ncclSuccess) {
                err = std::string("ncclGroupEnd: ") + ncclGetErrorString(r);
                return false;
            }
            return true;
        }
        for (int g = 0; g < G; ++g)
            if (!hip(hipSetDevice(dev[g]), "hipSetDevice") || !hip(hipEventRecord(ready[g], stream[g]), "hipEventRecord"))
                return false;
        for (int g = 0; g < G; ++g) {
            if (!hip(hipSetDevice(dev[g]), "hipSetDevice"))
                return false;
            for (int q = 0; q < G; ++q) {
                if (!hip(hipStreamWaitEvent(stream[g], ready[q], 0), "hipStreamWaitEvent") ||
                    !hip(hipMemcpyPeerAsync((char *)recv[g] + (size_t)q * bytes, dev[g], slot[q], dev[q], bytes,
                                            stream[g]),
                         "hipMemcpyPeerAsync"))
                    return false;
            }
        }
        return true;
    }
    ~Exchange()
    {
        // teardown: errors here have nowhere to go
        for (int g = 0; g < G; ++g) {
            (void)hipSetDevice(dev[g]);
            if (stream[g])
                (void)hipStreamSynchronize(stream[g]);
            if (rccl && g < (int)comm.size() && comm[g])
                ncclCommDestroy(comm[g]);
            if (slot[g])
                (void)hipFree(slot[g]);
            if (recv[g])
                (void)hipFree(recv[g]);
            if (ready[g])
                (void)hipEventDestroy(ready[g]);
            if (stream[g])
                (void)hipStreamDestroy(stream[g]);
        }
    }
};

// dp_densify over `ctxs.size()` contexts (one per GPU), the device-resident
// protocol of include/densepoints.h with ONE host wait per generation per
// context: every generation's items are partitioned by reference-view
// super-tile on the device (dp_densify_partition_async; the shares are
// host-known floor cuts), each context refines its share and compacts the
// accepted candidates into its slot (dp_densify_refine_share_async), the slots
// are all-gathered device to device (Exchange: RCCL or peer copies), and every
// context commits the whole generation to its replicated organizer
// (dp_densify_commit_gathered_device, in its own host thread so the waits
// overlap) -- no candidate touches host memory, and the store equals
// dp_densify's bit for bit.  Expansion generations of fewer than
// replicate_below items run on every context device-resident instead
// (dp_densify_run_until: no partition, no exchange, eight per host wait).
// Returns the stats of context 0 (evals / refine_ms summed / maxed).
int densify_multi(std::vector<dp_ctx *> &ctxs, const std::vector<int> &devices, const char *exchange_mode,
                  const std::vector<double> &seeds, std::vector<dp_patch> &out, dp_densify_stats &st,
                  std::string &err, int64_t &exchanged, int64_t replicate_below)
{
    const int G = (int)ctxs.size();
    const int n = (int)(seeds.size() / 3);
    Exchange ex;
    if (!ex.init(devices, exchange_mode)) {
        err = ex.err;
        return DP_E_HIP;
    }
    std::vector<dp_generation> gen((size_t)G);
    std::vector<int> rcs((size_t)G, DP_OK);
    auto fail_of = [&](int g, int rc) {
        err = dp_last_error(ctxs[(size_t)g]);
        return rc;
    };
    for (int g = 0; g < G; ++g) {
        const int rc = dp_densify_begin(ctxs[(size_t)g], seeds.data(), n, &gen[(size_t)g]);
        if (rc != DP_OK)
            return fail_of(g, rc);
    }
    exchanged = 0;
    std::vector<int64_t> counts((size_t)G), ex_g((size_t)G, 0), repl_evals((size_t)G, 0);
    while (gen[0].items > 0) {
        const int per = gen[0].per_item;
        if (gen[0].index >= 1 && gen[0].items < replicate_below) {
            // the BFS's small generations (latency-bound refines) on every
            // context at once, device-resident, no exchange, until one reaches
            // the bound; their evaluations count once (context 0)
            std::vector<std::thread> th;
            for (int g = 0; g < G; ++g)
                th.emplace_back([&, g]() {
                    int64_t ev = 0;
                    rcs[(size_t)g] = dp_densify_run_until(ctxs[(size_t)g], &gen[(size_t)g], INT32_MAX, replicate_below, &ev);
                    repl_evals[(size_t)g] += ev;
                });
            for (auto &t : th)
                t.join();
            for (int g = 0; g < G; ++g)
                if (rcs[(size_t)g] != DP_OK)
                    return fail_of(g, rcs[(size_t)g]);
            continue;
        }
        // the partition and each context's share, queued (no host wait)
        int64_t stride = 1;
        for (int g = 0; g < G; ++g) {
            const int64_t *d_order = nullptr;
            int rc = dp_densify_partition_async(ctxs[(size_t)g], &gen[(size_t)g], G, 64, ex.stream[(size_t)g], &d_order,
                                                counts.data());
            if (rc != DP_OK)
                return fail_of(g, rc);
            if (g == 0) {
                stride = std::max<int64_t>(*std::max_element(counts.begin(), counts.end()) * per, 1);
                if (!ex.reserve(stride)) {
                    err = ex.err;
                    return DP_E_HIP;
                }
            }
            int64_t off = 0;
            for (int q = 0; q < g; ++q)
                off += counts[(size_t)q];
            rc = dp_densify_refine_share_async(ctxs[(size_t)g], &gen[(size_t)g], counts[(size_t)g] ? d_order + off : nullptr,
                                               counts[(size_t)g], ex.slot[(size_t)g], stride, ex.stream[(size_t)g]);
            if (rc != DP_OK)
                return fail_of(g, rc);
        }
        if (!ex.all_gather(stride)) {
            err = ex.err;
            return DP_E_HIP;
        }
        std::vector<std::thread> th;
        for (int g = 0; g < G; ++g)
            th.emplace_back([&, g]() {
                rcs[(size_t)g] = dp_densify_commit_gathered_device(ctxs[(size_t)g], &gen[(size_t)g], ex.recv[(size_t)g],
                                                                   stride, G, ex.stream[(size_t)g], &ex_g[(size_t)g]);
            });
        for (auto &t : th)
            t.join();
        for (int g = 0; g < G; ++g)
            if (rcs[(size_t)g] != DP_OK)
                return fail_of(g, rcs[(size_t)g]);
        exchanged += ex_g[0];
    }
    std::vector<dp_densify_stats> sts((size_t)G);
    const dp_patch *res = nullptr;
    int64_t np = 0;
    for (int g = G - 1; g >= 0; --g) {
        const int rc = dp_densify_result(ctxs[(size_t)g], &res, &np, &sts[(size_t)g]);
        if (rc != DP_OK)
            return fail_of(g, rc);
    }
    out.assign(res, res + np);
    st = sts[0];
    for (int g = 1; g < G; ++g) {
        st.evals += sts[(size_t)g].evals - repl_evals[(size_t)g];
        st.refine_ms = std::max(st.refine_ms, sts[(size_t)g].refine_ms);
    }
    return DP_OK;
}

} // namespace

int main(int argc, char **argv)
{
    std::string input, settings, output = "points.ply", seeds_path, synth, scene_dir;
    int device = 0, gpus = 1;
    bool force_multi = false;
    std::string exchange_mode = "auto";
    long long replicate_below = -1; // default 1024 x contexts
    long long max_pops = -1;
    int level = 0;
    bool check_only = false, do_filter = false, fast = false;
    int fast_iters = -1, fast_gradient = -1;
    dp_matcher_options mopt; // MatcherOptions defaults (matcher.h:21-32), ORB::create(40000)
    dp_default_matcher_options(&mopt);
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) {
                usage();
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "-i" || a == "--input") input = next();
        else if (a == "-s" || a == "--settings") settings = next();
        else if (a == "-o" || a == "--output") output = next();
        else if (a == "--seeds") seeds_path = next();
        else if (a == "--device") device = std::atoi(next().c_str());
        else if (a == "--gpus") gpus = std::atoi(next().c_str());
        else if (a == "--multi") force_multi = true;
        else if (a == "--replicate-below") replicate_below = std::atoll(next().c_str());
        else if (a == "--exchange") {
            exchange_mode = next();
            if (exchange_mode != "auto" && exchange_mode != "rccl" && exchange_mode != "copy") {
                std::fprintf(stderr, "densify: --exchange expects auto, rccl or copy\n");
                return 2;
            }
        }
        else if (a == "--max-pops") max_pops = std::atoll(next().c_str());
        else if (a == "--level") level = std::atoi(next().c_str());
        else if (a == "--filter") do_filter = true;
        else if (a == "--check-only") check_only = true;
        else if (a == "--features") mopt.n_features = std::atoi(next().c_str());
        else if (a == "--fast-threshold") mopt.fast_threshold = std::atoi(next().c_str());
        else if (a == "--epipolar-matching") mopt.epipolar_matching = 1;
        else if (a == "--matcher") {
            const std::string v = next();
            if (v == "knn")
                mopt.matcher_type = DP_MATCHER_KNN;
            else if (v == "flann")
                mopt.matcher_type = DP_MATCHER_FLANN;
            else {
                std::fprintf(stderr, "densify: --matcher expects knn or flann\n");
                return 2;
            }
        }
        else if (a == "--detector") {
            const std::string v = next();
            if (v == "orb")
                mopt.detector_type = DP_DETECTOR_ORB;
            else if (v == "akaze")
                mopt.detector_type = DP_DETECTOR_AKAZE;
            else {
                std::fprintf(stderr, "densify: --detector expects orb or akaze\n");
                return 2;
            }
        } else if (a == "--akaze-threshold") mopt.akaze_threshold = (float)std::atof(next().c_str());
        else if (a == "--mode") {
            const std::string m = next();
            if (m != "parity" && m != "fast") {
                usage();
                return 2;
            }
            fast = m == "fast";
        } else if (a == "--fast-iters") fast_iters = std::atoi(next().c_str());
        else if (a == "--fast-gradient") fast_gradient = std::atoi(next().c_str());
        else if (a == "--synthetic") synth = next();
        else if (a == "--write-scene") scene_dir = next();
        else if (a == "-h" || a == "--help") {
            usage();
            return 0;
        } else {
            usage();
            return 2;
        }
    }
    try {
        if (!synth.empty()) {
            if (scene_dir.empty())
                throw std::runtime_error("--synthetic needs --write-scene DIR");
            return write_synthetic(synth, scene_dir);
        }
        if (input.empty()) {
            usage();
            return 2;
        }
        const auto t0 = std::chrono::steady_clock::now();
        dp_options opt;
        dp_default_options(&opt);
        if (!settings.empty())
            apply_settings(dpio::parse_json(dpio::read_file(settings)), opt);
        if (max_pops >= 0)
            opt.max_pops = max_pops;
        const dpio::Scene sc = dpio::read_scene(input);
        std::vector<dpio::Image> imgs;
        std::vector<double> P;
        for (const dpio::SceneView &v : sc.views) {
            imgs.push_back(dpio::load_image(v.filename)); // PMVS::AddCamera -> View::Load
            P.insert(P.end(), v.P, v.P + 12);
        }
        const std::vector<double> seeds = seeds_path.empty() ? std::vector<double>() : dpio::read_seeds(seeds_path);
        if (check_only) {
            // parsed scene summary + FNV-1a of each decoded BGR8 image (no GPU)
            std::printf("{\"views\": %zu, \"width\": %d, \"height\": %d, \"seeds\": %zu, \"image_fnv\": [",
                        imgs.size(), imgs.empty() ? 0 : imgs[0].width, imgs.empty() ? 0 : imgs[0].height,
                        seeds.size() / 3);
            for (size_t v = 0; v < imgs.size(); ++v) {
                uint64_t h = 1469598103934665603ull;
                for (uint8_t b : imgs[v].bgr)
                    h = (h ^ b) * 1099511628211ull;
                std::printf("%s\"%016llx\"", v ? ", " : "", (unsigned long long)h);
            }
            std::printf("]}\n");
            return 0;
        }
        std::vector<dp_image> dimg(imgs.size());
        for (size_t v = 0; v < imgs.size(); ++v)
            dimg[v] = dp_image{imgs[v].width, imgs[v].height, 3 * imgs[v].width, 0, imgs[v].bgr.data()};
        dp_ctx *ctx = nullptr;
        int rc = dp_ctx_create(&opt, device, &ctx);
        if (rc != DP_OK) {
            std::fprintf(stderr, "densify: dp_ctx_create failed (%d)\n", rc);
            return 1;
        }
        auto check = [&](int r, const char *what) {
            if (r != DP_OK) {
                std::fprintf(stderr, "densify: %s failed (%d): %s\n", what, r, dp_last_error(ctx));
                dp_ctx_destroy(ctx);
                std::exit(1);
            }
        };
        check(dp_set_views(ctx, (int)imgs.size(), P.data(), dimg.data()), "dp_set_views");
        // --mode fast: dp_fast_options.densify on every context
        dp_fast_options fo;
        dp_default_fast_options(&fo);
        fo.densify = fast ? 1 : 0;
        if (fast_iters >= 0)
            fo.iters = fast_iters;
        if (fast_gradient >= 0)
            fo.gradient = fast_gradient;
        check(dp_set_fast_options(ctx, &fo), "dp_set_fast_options");
        if (level > 0) {
            // run on pyramid level L (cv::pyrDown^L on the device, P rows 0-1 / 2^L)
            check(dp_build_pyramid(ctx, level + 1), "dp_build_pyramid");
            check(dp_set_level(ctx, level), "dp_set_level");
        }
        // PMVS::InsertSeeds (pmvs.cpp:29-34): without --seeds the seeds come from
        // Matcher::GenerateSeeds on the device (level-0 views)
        std::vector<double> gen_seeds;
        dp_seed_stats sst;
        std::memset(&sst, 0, sizeof sst);
        if (seeds_path.empty()) {
            const double *xyz = nullptr;
            int64_t n = 0;
            check(dp_generate_seeds(ctx, &mopt, &xyz, &n, &sst), "dp_generate_seeds");
            gen_seeds.assign(xyz, xyz + 3 * n);
        }
        const std::vector<double> &use = seeds_path.empty() ? gen_seeds : seeds;
        const dp_patch *out = nullptr;
        int64_t n_out = 0;
        dp_densify_stats st;
        std::memset(&st, 0, sizeof st);
        std::vector<dp_patch> multi_out;
        int64_t exchanged = -1;
        if (gpus > 1 || force_multi) {
            // contexts 1..N-1 on the next devices (wrapping: several ranks may share a GPU)
            const int ndev = dp_device_count();
            std::vector<dp_ctx *> ctxs{ctx};
            std::vector<int> devices{device};
            // a failure on a secondary context reports THAT context's error and
            // releases every context created so far before exiting
            auto check_g = [&](int rc, dp_ctx *cg, const char *what) {
                if (rc == DP_OK)
                    return;
                std::fprintf(stderr, "densify: %s failed on context %zu (%d): %s\n", what, ctxs.size(), rc,
                             cg ? dp_last_error(cg) : "context not created");
                if (cg && (ctxs.empty() || ctxs.back() != cg))
                    dp_ctx_destroy(cg);
                for (dp_ctx *x : ctxs)
                    dp_ctx_destroy(x);
                std::exit(1);
            };
            for (int g = 1; g < gpus; ++g) {
                dp_ctx *cg = nullptr;
                const int dg = (device + g) % (ndev > 0 ? ndev : 1);
                check_g(dp_ctx_create(&opt, dg, &cg), cg, "dp_ctx_create");
                ctxs.push_back(cg);
                devices.push_back(dg);
                check_g(dp_set_views(cg, (int)imgs.size(), P.data(), dimg.data()), cg, "dp_set_views");
                check_g(dp_set_fast_options(cg, &fo), cg, "dp_set_fast_options");
                if (level > 0) {
                    check_g(dp_build_pyramid(cg, level + 1), cg, "dp_build_pyramid");
                    check_g(dp_set_level(cg, level), cg, "dp_set_level");
                }
            }
            std::string err;
            const int64_t rb = replicate_below >= 0 ? (int64_t)replicate_below : 1024 * (int64_t)gpus;
            const int mrc =
                densify_multi(ctxs, devices, exchange_mode.c_str(), use, multi_out, st, err, exchanged, rb);
            for (int g = 1; g < gpus; ++g)
                dp_ctx_destroy(ctxs[(size_t)g]);
            if (mrc != DP_OK) {
                std::fprintf(stderr, "densify: multi-GPU densify failed (%d): %s\n", mrc, err.c_str());
                dp_ctx_destroy(ctx);
                return 1;
            }
            out = multi_out.data();
            n_out = (int64_t)multi_out.size();
        } else {
            check(dp_densify(ctx, use.data(), (int)(use.size() / 3), &out, &n_out, &st), "dp_densify");
        }
        // PMVS::FilterPatches (pmvs.h:27, undefined in the reference): dp_filter_patches spec
        std::vector<uint8_t> keep((size_t)n_out, 1);
        if (do_filter && n_out > 0) {
            dp_filter_options fo;
            dp_default_filter_options(&fo);
            check(dp_filter_patches(ctx, out, n_out, &fo, keep.data()), "dp_filter_patches");
        }
        std::vector<dpio::CloudPoint> cloud;
        cloud.reserve((size_t)n_out);
        for (int64_t i = 0; i < n_out; ++i) {
            if (!keep[i])
                continue;
            dpio::CloudPoint cp;
            for (int k = 0; k < 3; ++k) {
                cp.pos[k] = out[i].pos[k];
                cp.normal[k] = out[i].normal[k];
                cp.rgb[k] = out[i].rgb[k];
            }
            cloud.push_back(cp);
        }
        dp_ctx_destroy(ctx);
        dpio::write_ply(output, cloud);
        const double wall =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"output\": \"%s\", \"patches\": %lld, \"written\": %zu, \"seeds\": %zu, \"generated_seeds\": %s, "
                    "\"keypoints\": %lld, \"matches\": %lld, \"seed_ms\": %.3f, \"seed_patches\": %lld, "
                    "\"pops\": %lld, \"candidates\": %lld, \"evals\": %lld, \"generations\": %d, \"refine_ms\": %.3f, "
                    "\"densify_ms\": %.3f, \"wall_ms\": %.3f, \"gpus\": %d, \"mode\": \"%s\", \"exchanged\": %lld}\n",
                    output.c_str(), (long long)st.patches, cloud.size(), use.size() / 3,
                    seeds_path.empty() ? "true" : "false", (long long)sst.keypoints, (long long)sst.matches,
                    sst.total_ms, (long long)st.seed_patches, (long long)st.pops, (long long)st.candidates,
                    (long long)st.evals, st.generations, st.refine_ms, st.total_ms, wall, gpus,
                    fast ? "fast" : "parity", (long long)exchanged);
        return 0;
    } catch (const std::exception &e) {
        std::fprintf(stderr, "densify: %s\n", e.what());
        return 1;
    }
}
