// valu_probe.hip -- issue cost of the VALU instructions the performance-mode
// sampler uses, per SIMD, with 1 and 4 waves per SIMD (16 per CU).  Each wave
// runs REP x 32 independent copies of one instruction (8 accumulators) and
// reads the shader clock around the loop.  Build: hipcc --offload-arch=gfx950
// -O3 tools/valu_probe.hip -o /tmp/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define REP 256

#define BODY8(ins)                                                                                                     \
    asm volatile(ins : "+v"(a0) : "v"(b), "v"(c));                                                                     \
    asm volatile(ins : "+v"(a1) : "v"(b), "v"(c));                                                                     \
    asm volatile(ins : "+v"(a2) : "v"(b), "v"(c));                                                                     \
    asm volatile(ins : "+v"(a3) : "v"(b), "v"(c));                                                                     \
    asm volatile(ins : "+v"(a4) : "v"(b), "v"(c));                                                                     \
    asm volatile(ins : "+v"(a5) : "v"(b), "v"(c));                                                                     \
    asm volatile(ins : "+v"(a6) : "v"(b), "v"(c));                                                                     \
    asm volatile(ins : "+v"(a7) : "v"(b), "v"(c));

#define KERNEL(name, T, ins)                                                                                           \
    __global__ __launch_bounds__(64) void name(unsigned long long *out, T b, T c)                                      \
    {                                                                                                                  \
        T a0 = b, a1 = c, a2 = b, a3 = c, a4 = b, a5 = c, a6 = b, a7 = c;                                              \
        const unsigned long long t0 = __builtin_readcyclecounter();                                                   \
        for (int i = 0; i < REP; ++i) {                                                                                \
            BODY8(ins) BODY8(ins) BODY8(ins) BODY8(ins)                                                                \
        }                                                                                                              \
        const unsigned long long t1 = __builtin_readcyclecounter();                                                   \
        T s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                                                   \
        if (threadIdx.x == 0)                                                                                          \
            out[blockIdx.x] = (t1 - t0) + (s == (T)12345 ? 1 : 0);                                                     \
    }

KERNEL(k_fma_f32, float, "v_fma_f32 %0, %1, %2, %0")
KERNEL(k_add_u32, unsigned, "v_add_u32 %0, %1, %0")
KERNEL(k_mul_u24, unsigned, "v_mul_u32_u24 %0, %1, %0")
KERNEL(k_mad_u24, unsigned, "v_mad_u32_u24 %0, %1, %2, %0")
KERNEL(k_mul_lo_u32, unsigned, "v_mul_lo_u32 %0, %1, %0")
KERNEL(k_dot2_u16, unsigned, "v_dot2_u32_u16 %0, %1, %2, %0")
KERNEL(k_alignbit, unsigned, "v_alignbit_b32 %0, %1, %0, %2")
KERNEL(k_med3_f32, float, "v_med3_f32 %0, %1, %2, %0")
KERNEL(k_rcp_f32, float, "v_rcp_f32 %0, %0")
KERNEL(k_bfe_u32, unsigned, "v_bfe_u32 %0, %0, 5, 17")
KERNEL(k_add3_u32, unsigned, "v_add3_u32 %0, %1, %2, %0")
KERNEL(k_pk_fma_f32, double, "v_pk_fma_f32 %0, %1, %2, %0")
KERNEL(k_fma_f64, double, "v_fma_f64 %0, %1, %2, %0")
KERNEL(k_add_f64, double, "v_add_f64 %0, %1, %0")
KERNEL(k_dpp_add, unsigned, "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
KERNEL(k_cndmask, unsigned, "v_cndmask_b32_e64 %0, %0, %1, vcc")
KERNEL(k_mul_sdwa, unsigned, "v_mul_u32_u24_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1")
KERNEL(k_lshr, unsigned, "v_lshrrev_b32 %0, 4, %0")
KERNEL(k_rcp_f64, double, "v_rcp_f64 %0, %0")
KERNEL(k_rsq_f64, double, "v_rsq_f64 %0, %0")
KERNEL(k_sqrt_f64, double, "v_sqrt_f64 %0, %0")
KERNEL(k_div_fixup_f64, double, "v_div_fixup_f64 %0, %1, %2, %0")
KERNEL(k_ldexp_f64, double, "v_ldexp_f64 %0, %0, 3")
KERNEL(k_mul_f64, double, "v_mul_f64 %0, %1, %0")


typedef void (*kfn)(unsigned long long *, float, float);

template <typename T> static void run(const char *name, void (*k)(unsigned long long *, T, T), T b, T c, int cus)
{
    unsigned long long *d;
    const int maxb = cus * 16;
    hipMalloc(&d, sizeof(unsigned long long) * maxb);
    std::vector<unsigned long long> h(maxb);
    printf("%-14s", name);
    for (int wps : {1, 2, 4}) {
        const int nb = cus * 4 * wps;
        hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, d, b, c); // warm
        hipDeviceSynchronize();
        hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, d, b, c);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), d, sizeof(unsigned long long) * nb, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < nb; ++i)
            s += (double)h[i];
        s /= nb;
        // cycles per instruction per wave; per SIMD = that / waves per SIMD
        const double per_wave = s / (REP * 32.0);
        printf("  %d w/SIMD: %6.2f cyc/instr/wave %6.2f cyc/instr/SIMD", wps, per_wave, per_wave / wps);
    }
    printf("\n");
    hipFree(d);
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    run("fma_f32", k_fma_f32, 1.0001f, 0.5f, cus);
    run("add_u32", k_add_u32, 3u, 5u, cus);
    run("mul_u32_u24", k_mul_u24, 3u, 5u, cus);
    run("mad_u32_u24", k_mad_u24, 3u, 5u, cus);
    run("mul_lo_u32", k_mul_lo_u32, 3u, 5u, cus);
    run("dot2_u32_u16", k_dot2_u16, 3u, 5u, cus);
    run("alignbit", k_alignbit, 3u, 5u, cus);
    run("med3_f32", k_med3_f32, 1.0f, 2.0f, cus);
    run("rcp_f32", k_rcp_f32, 1.5f, 2.0f, cus);
    run("bfe_u32", k_bfe_u32, 3u, 5u, cus);
    run("add3_u32", k_add3_u32, 3u, 5u, cus);
    run("pk_fma_f32", k_pk_fma_f32, 1.0, 2.0, cus);
    run("fma_f64", k_fma_f64, 1.0, 0.5, cus);
    run("add_f64", k_add_f64, 1.0, 0.5, cus);
    run("add_u32_dpp", k_dpp_add, 3u, 5u, cus);
    run("cndmask", k_cndmask, 3u, 5u, cus);
    run("mul_u24_sdwa", k_mul_sdwa, 3u, 5u, cus);
    run("lshrrev", k_lshr, 3u, 5u, cus);
    run("rcp_f64", k_rcp_f64, 1.5, 2.0, cus);
    run("rsq_f64", k_rsq_f64, 1.5, 2.0, cus);
    run("sqrt_f64", k_sqrt_f64, 1.5, 2.0, cus);
    run("div_fixup_f64", k_div_fixup_f64, 1.5, 2.0, cus);
    run("ldexp_f64", k_ldexp_f64, 1.5, 2.0, cus);
    run("mul_f64", k_mul_f64, 1.0001, 2.0, cus);
    return 0;
}
