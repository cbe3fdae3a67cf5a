// batch_mask_device.h -- the mask statistics of a sampled learner batch, computed by one workgroup of the REFIL
// learner's prologue launch (refil_learner.hip prologue_kernel; replaces its three serial per-episode scans, whose
// dependent loads made block 0 the launch's longest task; the QMIX learner's prep_kernel keeps its two-pass
// mask_sum_block, measured 2 us faster there, profiles/r06/s16_mask_stats_ab/). Restates the reference's mask and
// truncation (q_learner.py:58-60, 89-95; ma_experiment.py:235-239):
//   mask(b, t) = filled(b, t) * (1 - terminated(b, t - 1))   (t > 0; t = 0: filled(b, 0))
//   Te         = clamp(max_b sum_t filled(b, t), 2, T)           (max_t_filled)
//   msum[0]    = sum_{b, t < Te - 1} mask(b, t),  msum[1] = Te
//   mixlen[b]  = 1 + the last t < Te - 1 with mask(b, t) != 0    (0: none; REFIL only)
// One pass of independent loads over the B x T elements (a thread per element, EPT elements in flight per thread),
// the per-episode filled counts and live bits gathered with LDS atomics, then a thread per episode. Every quantity is
// an integer count (exact in float), so the results equal the serial per-episode scans bit for bit. The lds buffer
// holds B <= MLG_MS_BMAX episodes of T <= 32 * MLG_MS_TW steps (callers fall back to their scans otherwise).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mlg {

constexpr int MLG_MS_BMAX = 256, MLG_MS_TW = 4;

struct MaskStatsLds {
    int cnt[MLG_MS_BMAX];                 // filled steps per episode
    uint32_t live[MLG_MS_BMAX][MLG_MS_TW];  // mask(b, t) != 0 as bits
    int te, total;
};

__host__ __device__ constexpr bool mask_stats_fits(int B, int T) { return B <= MLG_MS_BMAX && T <= 32 * MLG_MS_TW; }

// slot(b): the episode's row in the batch storage (sampled views)
template <class SlotFn>
__device__ void batch_mask_stats(const int64_t* __restrict__ filled, const uint8_t* __restrict__ term, int T1,
                                 SlotFn slot, int B, int T, float* __restrict__ msum, float* __restrict__ mixlen,
                                 MaskStatsLds& S) {
    constexpr int EPT = 4;
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int b = tid; b < B; b += nt) {
        S.cnt[b] = 0;
#pragma unroll
        for (int w = 0; w < MLG_MS_TW; ++w) S.live[b][w] = 0u;
    }
    if (tid == 0) S.te = S.total = 0;
    __syncthreads();
    const int n = B * T;
    for (int i0 = tid; i0 < n; i0 += EPT * nt) {
        int64_t f[EPT];
        uint8_t tp[EPT];
        int bb[EPT], tt[EPT];
#pragma unroll
        for (int k = 0; k < EPT; ++k) {  // every load of the group issued before any is used
            const int i = i0 + k * nt;
            const bool in = i < n;
            const int b = in ? i / T : 0, t = in ? i - b * T : 0;
            const int64_t base = slot(b) * T1;
            bb[k] = in ? b : -1;
            tt[k] = t;
            f[k] = in ? filled[base + t] : 0;
            tp[k] = (in && t > 0) ? term[base + t - 1] : (uint8_t)0;
        }
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            if (bb[k] < 0 || f[k] == 0) continue;
            atomicAdd(&S.cnt[bb[k]], 1);
            if (tp[k] == 0) atomicOr(&S.live[bb[k]][tt[k] >> 5], 1u << (tt[k] & 31));
        }
    }
    __syncthreads();
    for (int b = tid; b < B; b += nt) atomicMax(&S.te, S.cnt[b]);
    __syncthreads();
    const int Te = min(max(S.te, 2), T);
    for (int b = tid; b < B; b += nt) {
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
