// batch_mask_device.h -- the mask statistics of a sampled learner batch, computed by one workgroup of a learner's
// prologue launch (learner.hip prep_kernel block 0, refil_learner.hip prologue_kernel block 0). Restates the
// reference's mask and truncation (q_learner.py:58-60, 89-95; ma_experiment.py:235-239):
//   mask(b, t) = filled(b, t) * (1 - terminated(b, t - 1))   (t > 0; t = 0: filled(b, 0))
//   Te         = clamp(max_b sum_t filled(b, t), 2, T)           (max_t_filled)
//   msum[0]    = sum_{b, t < Te - 1} mask(b, t),  msum[1] = Te
//   mixlen[b]  = 1 + the last t < Te - 1 with mask(b, t) != 0    (0: none; REFIL only)
// A wave per episode (episodes wave, wave + waves, ... up to EPW per wave) with every load of all of the wave's
// episodes issued before the first is used -- one memory round trip, where the serial per-episode scans it replaces
// waited once per episode and 64-step chunk -- then ballots: each episode's filled count and live bits are written
// by one lane (no atomics on shared counters), Te is one atomicMax per episode. Every quantity is an integer count
// (exact in float), so the results equal the scans bit for bit. Holds B <= waves * EPW episodes of T <= 32 *
// MLG_MS_TW steps (mask_stats_fits; callers fall back to their scans otherwise).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mlg {

constexpr int MLG_MS_BMAX = 256, MLG_MS_TW = 4;

struct MaskStatsLds {
    int cnt[MLG_MS_BMAX];                   // filled steps per episode
    uint32_t live[MLG_MS_BMAX][MLG_MS_TW];  // mask(b, t) != 0 as bits
    int te, total;
};

template <int EPW>
__host__ __device__ constexpr bool mask_stats_fits(int B, int T, int waves) {
    return B <= MLG_MS_BMAX && B <= waves * EPW && T <= 32 * MLG_MS_TW;
}

// slot(b): the episode's row in the batch storage (sampled views)
template <int EPW, class SlotFn>
__device__ void batch_mask_stats(const int64_t* __restrict__ filled, const uint8_t* __restrict__ term, int T1,
                                 SlotFn slot, int B, int T, float* __restrict__ msum, float* __restrict__ mixlen,
                                 MaskStatsLds& S) {
    static_assert(MLG_MS_TW == 4, "two 64-step chunks per episode");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    if (tid == 0) S.te = S.total = 0;
    int64_t f[EPW][2];
    uint8_t tp[EPW][2];
#pragma unroll
    for (int k = 0; k < EPW; ++k) {  // every load of the wave's episodes before the first use
        const int b = wave + nw * k;
        const bool eb = b < B;
        const int64_t base = slot(eb ? b : 0) * T1;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int t = 64 * c + lane;
            const bool in = eb && t < T;
            f[k][c] = in ? filled[base + t] : 0;
            tp[k][c] = (in && t > 0) ? term[base + t - 1] : (uint8_t)0;
        }
    }
    __syncthreads();  // te / total initialised
#pragma unroll
    for (int k = 0; k < EPW; ++k) {
        const int b = wave + nw * k;
        if (b >= B) break;  // wave-uniform
        const uint64_t f0 = __ballot(f[k][0] != 0), f1 = __ballot(f[k][1] != 0);
        const uint64_t l0 = __ballot(f[k][0] != 0 && tp[k][0] == 0), l1 = __ballot(f[k][1] != 0 && tp[k][1] == 0);
        if (lane == 0) {
            const int n = __popcll(f0) + __popcll(f1);
            S.cnt[b] = n;
            S.live[b][0] = (uint32_t)l0;
            S.live[b][1] = (uint32_t)(l0 >> 32);
            S.live[b][2] = (uint32_t)l1;
            S.live[b][3] = (uint32_t)(l1 >> 32);
            atomicMax(&S.te, n);
        }
    }
    __syncthreads();
    const int Te = min(max(S.te, 2), T);
    for (int b = tid; b < B; b += blockDim.x) {
        int c = 0, last = -1;
#pragma unroll
        for (int w = 0; w < MLG_MS_TW; ++w) {
            const int lim = Te - 1 - 32 * w;  // steps t < Te - 1 of this word
            const uint32_t keep = lim >= 32 ? 0xFFFFFFFFu : (lim <= 0 ? 0u : ((1u << lim) - 1u));
            const uint32_t m = S.live[b][w] & keep;
            c += __builtin_popcount(m);
            if (m) last = 32 * w + 31 - __builtin_clz(m);
        }
        if (c) atomicAdd(&S.total, c);
        if (mixlen) mixlen[b] = (float)(last + 1);
    }
    __syncthreads();
    if (tid == 0) {
        msum[0] = (float)S.total;
        msum[1] = (float)Te;
    }
}

}  // namespace mlg
