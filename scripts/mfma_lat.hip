// Latency / issue microbenchmark for the learner recurrences' building blocks on gfx950 (one block, 4 waves):
// chains of dependent v_mfma_f32_4x4x1_16b_f32 / 16x16x4 f32 / 16x16x32 bf16, cross-lane exchanges and the
// workgroup barrier. Prints shader-clock cycles per operation and the shader clock (vs s_memrealtime, 100 MHz).
// Build: hipcc --offload-arch=gfx950 -O3 scripts/mfma_lat.hip -o scripts/mfma_lat
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int ITERS = 2000;

template <int MODE, int CH>
__global__ void __launch_bounds__(256) bench(float* out, unsigned long long* cyc, float seed) {
    floatx4 acc[CH];
    for (int c = 0; c < CH; ++c) acc[c] = floatx4{seed, 0.f, 0.f, (float)c};
    float a = seed * (1.f + threadIdx.x), b = seed * 2.f;
    bf16x8 av, bv;
    for (int i = 0; i < 8; ++i) {
        av[i] = (__bf16)(a + i);
        bv[i] = (__bf16)(b - i);
    }
    float x = seed + threadIdx.x;
    __shared__ float lds[256];
    lds[threadIdx.x] = x;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if constexpr (MODE == 0) acc[c] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[c], 0, 0, 0);
                if constexpr (MODE == 1) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
                if constexpr (MODE == 2) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[c], 0, 0, 0);
            }
            if constexpr (MODE == 3) x = __shfl(x, (threadIdx.x + 16) & 63, 64) * 1.0001f;
            if constexpr (MODE == 4) {
                const unsigned u = __float_as_uint(x);
                x = __uint_as_float(__builtin_amdgcn_permlane16_swap(u, u, false, false)[1]) * 1.0001f;
            }
            if constexpr (MODE == 5) {
                lds[threadIdx.x] = x;
                __syncthreads();
                x = lds[(threadIdx.x + 64) & 255] * 1.0001f;
            }
            if constexpr (MODE == 6) {
                lds[threadIdx.x] = x;
                x = lds[(threadIdx.x + 1) & 255] * 1.0001f;
            }
            if constexpr (MODE == 7) x = 1.f / (1.f + __builtin_amdgcn_exp2f(-x * 1.4426950f));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = x;
    for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = r1 - r0;
    }
}

template <int MODE, int CH>
void run(const char* name, float* d_out, unsigned long long* d_cyc, float seed = 1.0f) {
    hipLaunchKernelGGL((bench<MODE, CH>), dim3(1), dim3(256), 0, 0, d_out, d_cyc, seed);
    hipLaunchKernelGGL((bench<MODE, CH>), dim3(1), dim3(256), 0, 0, d_out, d_cyc, seed);
    unsigned long long h[2];
    hipMemcpy(h, d_cyc, sizeof(h), hipMemcpyDeviceToHost);
    const double ops = (double)ITERS * 8 * (MODE <= 2 ? CH : 1);
    printf("%-34s chains=%d  cycles/op=%7.2f  (per op, all chains) ns/op=%7.2f  clock=%.0f MHz\n", name, CH,
           h[0] / ops, h[1] * 10.0 / ops, h[0] * 100.0 / h[1]);
}

int main() {
    float* d_out;
    unsigned long long* d_cyc;
    hipMalloc(&d_out, 256 * sizeof(float));
    hipMalloc(&d_cyc, 2 * sizeof(unsigned long long));
    run<0, 1>("mfma 4x4x1 f32", d_out, d_cyc);
    run<0, 2>("mfma 4x4x1 f32", d_out, d_cyc);
    run<0, 2>("mfma 4x4x1 f32 (nan operands)", d_out, d_cyc, __builtin_nanf(""));
    run<0, 2>("mfma 4x4x1 f32 (denormal operands)", d_out, d_cyc, 1e-39f);
    run<0, 2>("mfma 4x4x1 f32 (zero operands)", d_out, d_cyc, 0.f);
    run<0, 4>("mfma 4x4x1 f32", d_out, d_cyc);
    run<0, 8>("mfma 4x4x1 f32", d_out, d_cyc);
    run<1, 1>("mfma 16x16x4 f32", d_out, d_cyc);
    run<1, 4>("mfma 16x16x4 f32", d_out, d_cyc);
    run<2, 1>("mfma 16x16x32 bf16", d_out, d_cyc);
    run<2, 4>("mfma 16x16x32 bf16", d_out, d_cyc);
    run<3, 1>("ds_bpermute round trip", d_out, d_cyc);
    run<4, 1>("permlane16_swap round trip", d_out, d_cyc);
    run<5, 1>("lds write+barrier+read (4 waves)", d_out, d_cyc);
    run<6, 1>("lds write+wait+read", d_out, d_cyc);
    run<7, 1>("sigmoid (exp+rcp) chain", d_out, d_cyc);
    hipFree(d_out);
    hipFree(d_cyc);
    return 0;
}
