// Throughput of single VALU instruction classes on gfx950: every wave runs 8
// independent chains of the instruction for ITER iterations; reported as
// cycles per wave-instruction per SIMD (at the measured clock).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITER 4096
#define CHAINS 8

#define K(NAME, ASM)                                                                       \
    __global__ void NAME(uint32_t *out, uint32_t seed)                                     \
    {                                                                                      \
        uint32_t a[CHAINS];                                                                \
        uint32_t b = seed ^ threadIdx.x;                                                   \
        for (int c = 0; c < CHAINS; c++) a[c] = seed * (c + 1) + threadIdx.x;              \
        for (int i = 0; i < ITER; i++) {                                                   \
            _Pragma("unroll") for (int c = 0; c < CHAINS; c++) asm volatile(ASM : "+v"(a[c]) : "v"(b)); \
        }                                                                                  \
        uint32_t s = 0;                                                                    \
        for (int c = 0; c < CHAINS; c++) s += a[c];                                        \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                    \
    }

K(k_add_f32, "v_add_f32 %0, %0, %1")
K(k_mul_f32, "v_mul_f32 %0, %0, %1")
K(k_fma_f32, "v_fma_f32 %0, %0, %1, %0")
K(k_add_u32, "v_add_u32 %0, %0, %1")
K(k_xor_b32, "v_xor_b32 %0, %0, %1")
K(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
K(k_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
K(k_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
K(k_sqrt_f32, "v_sqrt_f32 %0, %0")
K(k_rcp_f32, "v_rcp_f32 %0, %0")
K(k_cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
K(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
K(k_alignbit, "v_alignbit_b32 %0, %0, %1, 7")
K(k_mov, "v_mov_b32 %0, %1")
K(k_cndmask_s, "s_mov_b64 s[40:41], 0x5555\n v_cndmask_b32_e64 %0, %0, %1, s[40:41]")
K(k_cmp_cnd, "v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc")
K(k_cmp_cnd_s, "v_cmp_lt_f32_e64 s[40:41], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[40:41]")
K(k_readfirst, "v_readfirstlane_b32 s40, %0\n v_add_u32 %0, s40, %0")
K(k_max3, "v_max3_f32 %0, %0, %1, %0")
K(k_med3, "v_med3_f32 %0, %0, %1, %0")

#define K64(NAME, ASM)                                                                     \
    __global__ void NAME(uint32_t *out, uint32_t seed)                                     \
    {                                                                                      \
        uint64_t a[CHAINS];                                                                \
        uint32_t b = seed ^ threadIdx.x;                                                   \
        uint64_t bb = ((uint64_t)b << 32) | (b * 3u);                                      \
        for (int c = 0; c < CHAINS; c++) a[c] = (uint64_t)seed * (c + 1) + threadIdx.x;    \
        for (int i = 0; i < ITER; i++) {                                                   \
            _Pragma("unroll") for (int c = 0; c < CHAINS; c++) asm volatile(ASM : "+v"(a[c]) : "v"(b), "v"(bb)); \
        }                                                                                  \
        uint64_t s = 0;                                                                    \
        for (int c = 0; c < CHAINS; c++) s += a[c];                                        \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);   \
    }

K64(k_mad_u64_u32, "v_mad_u64_u32 %0, vcc, %1, %1, %0")
K64(k_pk_add_f32, "v_pk_add_f32 %0, %0, %2")
K64(k_pk_mul_f32, "v_pk_mul_f32 %0, %0, %2")
K64(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %2, %0")
K64(k_lshl_b64, "v_lshlrev_b64 %0, 3, %0")
K64(k_add_f64, "v_add_f64 %0, %0, %2")

typedef void (*kfn)(uint32_t *, uint32_t);

int main()
{
    int dev = 0, cus = 0, clk = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    struct { const char *name; kfn f; } ks[] = {
        {"v_add_f32", k_add_f32}, {"v_mul_f32", k_mul_f32}, {"v_fma_f32", k_fma_f32}, {"v_add_u32", k_add_u32},
        {"v_xor_b32", k_xor_b32}, {"v_mul_lo_u32", k_mul_lo_u32}, {"v_mul_hi_u32", k_mul_hi_u32},
        {"v_mul_u32_u24", k_mul_u32_u24}, {"v_sqrt_f32", k_sqrt_f32}, {"v_rcp_f32", k_rcp_f32},
        {"v_cvt_f32_u32", k_cvt_f32_u32}, {"v_cndmask_b32", k_cndmask}, {"v_alignbit_b32", k_alignbit},
        {"v_mov_b32", k_mov}, {"s_mov+cndmask_e64", k_cndmask_s}, {"cmp+cndmask(vcc)", k_cmp_cnd},
        {"cmp+cndmask(sgpr)", k_cmp_cnd_s}, {"readfirstlane+add", k_readfirst}, {"v_max3_f32", k_max3}, {"v_med3_f32", k_med3}, {"v_mad_u64_u32", k_mad_u64_u32}, {"v_pk_add_f32", k_pk_add_f32},
        {"v_pk_mul_f32", k_pk_mul_f32}, {"v_pk_fma_f32", k_pk_fma_f32}, {"v_lshlrev_b64", k_lshl_b64},
        {"v_add_f64", k_add_f64},
    };
    const int waves_per_simd[] = {1, 2, 4};
    uint32_t *out;
    hipMalloc(&out, (size_t)cus * 16 * 64 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("CUs %d, clock %d kHz; cycles per wave-instruction per SIMD (nominal clock)\n", cus, clk);
    printf("%-16s %8s %8s %8s\n", "instr", "1w/SIMD", "2w/SIMD", "4w/SIMD");
    for (auto &k : ks) {
        printf("%-16s", k.name);
        for (int w : waves_per_simd) {
            int blocks = cus, threads = 64 * 4 * w; /* one block per CU, w waves per SIMD */
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1u);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 2u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            double cycles = ms * 1e-3 * clk * 1e3;
            double instr_per_simd = (double)ITER * CHAINS * w;
            printf(" %8.2f", cycles / instr_per_simd);
        }
        printf("\n");
    }
    return 0;
}
