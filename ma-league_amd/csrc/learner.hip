// learner.hip -- QLearner.train (src/marl/learners/q_learner.py:34-131) as one device pipeline on gfx950.
//
//   pack        online/target agent + mixer weights -> kernel layouts (+ W_ih^T for backward)
//   mask_sum    mask = filled[:, :-1] * (1 - terminated shifted) and its sum                (:36-42, :89-98)
//   agent_in    fc1 + W_ih x for every (t, row), online + target, fully parallel               (:44-65)
//   agent_rec   the recurrence only (W_hh h + gates), one workgroup per 16 sequence rows,
//               wave w owns hidden chunk w with its W_hh rows in VGPRs; saves gates
//   agent_q     fc2 for every (t, row), fully parallel
//   mix_td      per (b, t) row: gather chosen Q, double-Q target, QMixer fwd (online+target),
//               TD error, masked MSE partials, QMixer backward -> dQ and mixer deltas         (:55-98)
//   agent_bwd   reverse-time GRU backward (dh carried in registers, dGH exchanged in LDS)    (:103)
//   agent_dx    dX = W_ih^T dGI * relu' for every (t, row), fully parallel
//   wgrad       every weight/bias gradient as sum_rows delta^T x, one wave per 64x64 block and row chunk
//               (deterministic slab reduction; MFMA with the row index as K)
//   finish      loss/stat reduction, clip_grad_norm_(10), RMSprop step                       (:104-105, learner.py:25-31)
// Tensors saved for backward are t-major: [T][R][F] with R = B * N agent rows (r = b * N + n).
#include <algorithm>

#include "agent_device.h"
#include "batch_mask_device.h"
#include "gru4_device.h"
#include "mlg_host.h"
#include "wgrad_device.h"

namespace {

using WJobs = mlg::BJobsT<16>;
using mlg::WJob;
using mlg::job;
using mlg::block_sum_1024;

// ---- canonical flat parameter offsets (nn.Module named_parameters order) ------------------------
struct AgentOffs {
    int64_t fc1w, fc1b, wih, whh, bih, bhh, fc2w, fc2b, total;
};
__host__ __device__ inline AgentOffs agent_offs(int H, int d_in, int A) {
    AgentOffs o;
    int64_t p = 0;
    o.fc1w = p; p += (int64_t)H * d_in;
    o.fc1b = p; p += H;
    o.wih = p; p += (int64_t)3 * H * H;
    o.whh = p; p += (int64_t)3 * H * H;
    o.bih = p; p += 3 * H;
    o.bhh = p; p += 3 * H;
    o.fc2w = p; p += (int64_t)A * H;
    o.fc2b = p; p += A;
    o.total = p;
    return o;
}

struct MixOffs {
    int64_t w1_0w, w1_0b, w1_2w, w1_2b, wf_0w, wf_0b, wf_2w, wf_2b, b1w, b1b, v0w, v0b, v2w, v2b, total;
};
__host__ __device__ inline MixOffs mix_offs(int N, int S, int E, int HE) {
    MixOffs o;
    int64_t p = 0;
    o.w1_0w = p; p += (int64_t)HE * S;
    o.w1_0b = p; p += HE;
    o.w1_2w = p; p += (int64_t)N * E * HE;
    o.w1_2b = p; p += (int64_t)N * E;
    o.wf_0w = p; p += (int64_t)HE * S;
    o.wf_0b = p; p += HE;
    o.wf_2w = p; p += (int64_t)E * HE;
    o.wf_2b = p; p += E;
    o.b1w = p; p += (int64_t)E * S;
    o.b1b = p; p += E;
    o.v0w = p; p += (int64_t)E * S;
    o.v0b = p; p += E;
    o.v2w = p; p += E;
    o.v2b = p; p += 1;
    o.total = p;
    return o;
}

// ---- packed mixer block: m1 = [w1h | wfh | b1 | vh] rows over padded state, transposes, padded V.2 ----
struct MixPack {
    int L1, Sp, NE;
    int64_t m1, mb1, a2T, f2T, v2p, bv2p, total;
};
__host__ __device__ inline MixPack mix_pack(int N, int S, int E, int HE) {
    MixPack m;
    m.L1 = 2 * HE + 2 * E;
    m.Sp = (S + 15) / 16 * 16;
    m.NE = N * E;
    int64_t p = 0;
    m.m1 = p; p += (int64_t)m.L1 * m.Sp;
    m.mb1 = p; p += m.L1;
    m.a2T = p; p += (int64_t)HE * m.NE;
    m.f2T = p; p += (int64_t)HE * E;
    m.v2p = p; p += (int64_t)16 * E;
    m.bv2p = p; p += 16;
    m.total = mlg_align4(p);
    return m;
}

struct MixPtrs {
    const float *m1, *mb1, *a2, *ba2, *a2T, *f2, *bf2, *f2T, *v2p, *bv2p;
};

// ---- device config ---------------------------------------------------------------------------------
struct LCfg {
    int B, T, T1, N, A, Ap, d_obs, d_in, H, S, E, HE, mixer, double_q, last_action, agent_id;
    int R, RM;
    float gamma;
};

// ---- workspace layout --------------------------------------------------------------------------------
struct WsLayout {
    int64_t p_on, p_tg, wihT, mix_on, mix_tg;
    int64_t in, x, hs, hs_tg, gi_on, gi_tg, gr, gz, gn, ghn, mac, tmac, dq, d2, dgi, dgh, da;
    int64_t srow, l1act, d1, da2, df2, dv2, hyp_on, hyp_tg;
    int64_t part, msum, rows, nrm, slab, total;
    int n_mix_tiles, n_tasks, hyp_stride;
};

__host__ __device__ inline int64_t a4(int64_t v) { return mlg_align4(v); }

// ================================================================================================
// packing
__device__ __forceinline__ float pack_mixer_elem(const MixPack& mp, const MixOffs& mo, const float* __restrict__ P,
                                                 int64_t i, int S, int E, int HE) {
    float v = 0.f;
    if (i < mp.mb1) {
        const int r = (int)(i / mp.Sp), c = (int)(i % mp.Sp);
        if (c < S) {
            if (r < HE) v = P[mo.w1_0w + (int64_t)r * S + c];
            else if (r < 2 * HE) v = P[mo.wf_0w + (int64_t)(r - HE) * S + c];
            else if (r < 2 * HE + E) v = P[mo.b1w + (int64_t)(r - 2 * HE) * S + c];
            else v = P[mo.v0w + (int64_t)(r - 2 * HE - E) * S + c];
        }
    } else if (i < mp.a2T) {
        const int r = (int)(i - mp.mb1);
        if (r < HE) v = P[mo.w1_0b + r];
        else if (r < 2 * HE) v = P[mo.wf_0b + r - HE];
        else if (r < 2 * HE + E) v = P[mo.b1b + r - 2 * HE];
        else v = P[mo.v0b + r - 2 * HE - E];
    } else if (i < mp.f2T) {  // a2T [HE][NE] = w1_2w^T
        const int64_t k = i - mp.a2T;
        const int r = (int)(k / mp.NE), c = (int)(k % mp.NE);
        v = P[mo.w1_2w + (int64_t)c * HE + r];
    } else if (i < mp.v2p) {  // f2T [HE][E]
        const int64_t k = i - mp.f2T;
        const int r = (int)(k / E), c = (int)(k % E);
        v = P[mo.wf_2w + (int64_t)c * HE + r];
    } else if (i < mp.bv2p) {  // v2p [16][E], row 0 = V.2.weight
        const int64_t k = i - mp.v2p;
        if (k < E) v = P[mo.v2w + k];
    } else if (i < mp.bv2p + 16) {
        if (i == mp.bv2p) v = P[mo.v2b];
    }
    return v;
}

// episode b of the batch -> its slot in the tensors (sampled view of the replay buffer: rows[b])
__device__ __forceinline__ int64_t bslot(const MlgBatch& bt, int b) { return bt.rows ? (int64_t)bt.rows[b] : (int64_t)b; }

// ================================================================================================
// mask: mask[b][t] = filled[b][t] * (t > 0 ? 1 - terminated[b][t-1] : 1), t < T-1
__device__ __forceinline__ float mask_at(const MlgBatch& bt, int b, int t) {
    const int64_t base = bslot(bt, b) * bt.T1;
    float m = (float)bt.filled[base + t];
    if (t > 0) m *= 1.f - (float)bt.terminated[base + t - 1];
    return m;
}

// One 1024-thread block: sum of the mask and max_t_filled (msum[0], msum[1]).
__device__ void mask_sum_block(const MlgBatch& bt, int B, int T, float* __restrict__ msum, float* red) {
    // msum[1] = max_t_filled (the reference's truncation, ma_experiment.py:235-239): the learner uses transitions
    // t < max_t_filled - 1 only; the sequential kernels stop there and the per-t kernels skip the steps beyond
    int mx = 0;  // a wave per episode: filled steps counted with ballots
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int b = wave; b < B; b += nw) {
        const int64_t base = bslot(bt, b) * bt.T1;
        int n = 0;
        for (int t0 = 0; t0 < T; t0 += 64) {
            const int t = t0 + lane;
            n += __popcll(__ballot(t < T && bt.filled[base + t] != 0));
        }
        mx = n > mx ? n : mx;
    }
    red[threadIdx.x] = (float)mx;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    const int Te = (int)fminf(fmaxf(red[0], 2.f), (float)T);
    __syncthreads();
    float s = 0.f;
    for (int i = threadIdx.x; i < B * (Te - 1); i += blockDim.x) s += mask_at(bt, i / (Te - 1), i % (Te - 1));
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        msum[0] = red[0];
        msum[1] = (float)Te;
    }
}

// Fused learner prologue (one launch instead of eight): block 0 sums the mask (mask_sum_block); the other blocks
// pack the online / target agent weights (pack_agent_elem), transpose W_ih (dX pass), pack the online / target
// QMixer hypernets (pack_mixer_elem) and zero the sparse delta buffers d2 and dq.
struct PrepJob {
    AgentLayout L;
    MlgAgentParams ap_on, ap_tg;
    float *p_on, *p_tg;
    const float* wih;  // [3H][H] -> wihT [H][3H]
    float* wihT;
    int rows3, cols;
    MixPack mp;
    MixOffs mo;
    const float *mix_src_on, *mix_src_tg;
    float *mix_on, *mix_tg;
    int N, S, E, HE, mixer;
    float *d2, *dq;
    int64_t n_d2, n_dq;
    MlgBatch bt;
    int B, T;
    float* msum;
    int n_rows_in;          // > 0: the slot map travels here (host_rows); block 0 stores it to rows_dst
    int32_t* rows_dst;
    int32_t rows_in[MLG_INLINE_ROWS];
};
static_assert(sizeof(PrepJob) <= 3072, "PrepJob must fit the kernel-argument segment");

__global__ void __launch_bounds__(1024) prep_kernel(PrepJob J) {
    if (blockIdx.x == 0) {
        __shared__ float red[1024];
        __shared__ int32_t srows[MLG_INLINE_ROWS];
        __shared__ mlg::MaskStatsLds ms;
        MlgBatch b2 = J.bt;
        if (J.n_rows_in > 0) {  // the block reads the slot map from LDS; later launches from rows_dst
            if (threadIdx.x < J.n_rows_in) {
                srows[threadIdx.x] = J.rows_in[threadIdx.x];
                J.rows_dst[threadIdx.x] = J.rows_in[threadIdx.x];
            }
            __syncthreads();
            b2.rows = srows;
        }
        constexpr int EPW = 4;  // episodes per wave: 16 waves cover batches of up to 64 episodes
        if (mlg::mask_stats_fits<EPW>(J.B, J.T, blockDim.x / 64))  // one round trip (batch_mask_device.h)
            mlg::batch_mask_stats<EPW>(b2.filled, b2.terminated, b2.T1, [&](int b) { return bslot(b2, b); }, J.B, J.T,
                                       J.msum, nullptr, ms);
        else
            mask_sum_block(b2, J.B, J.T, J.msum, red);
        return;
    }
    const int64_t na = J.L.gsp,  // the learner reads no pre-split rollout sections (gsp, w1s)
                   nt = (int64_t)J.rows3 * J.cols, nm = J.mixer == 2 ? J.mp.total : 0;
    const int64_t total = 2 * na + nt + 2 * nm + J.n_d2 + J.n_dq;
    for (int64_t i = (int64_t)(blockIdx.x - 1) * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)(gridDim.x - 1) * blockDim.x) {
        int64_t k = i;
        if (k < na) { J.p_on[k] = pack_agent_elem(J.L, J.ap_on, k); continue; }
        k -= na;
        if (k < na) { J.p_tg[k] = pack_agent_elem(J.L, J.ap_tg, k); continue; }
        k -= na;
        if (k < nt) {  // wihT[c][r] = wih[r][c]
            const int r = (int)(k / J.cols), c = (int)(k % J.cols);
            J.wihT[(int64_t)c * J.rows3 + r] = J.wih[k];
            continue;
        }
        k -= nt;
        if (k < nm) { J.mix_on[k] = pack_mixer_elem(J.mp, J.mo, J.mix_src_on, k, J.S, J.E, J.HE); continue; }
        k -= nm;
        if (k < nm) { J.mix_tg[k] = pack_mixer_elem(J.mp, J.mo, J.mix_src_tg, k, J.S, J.E, J.HE); continue; }
        k -= nm;
        if (k < J.n_d2) { J.d2[k] = 0.f; continue; }
        k -= J.n_d2;
        J.dq[k] = 0.f;
    }
}


#ifdef MLG_STAMPS
// Diagnostic build only (-DMLG_STAMPS): per-wave cycle counts of the recurrences' step phases, written to
// g_mlg_lstamps[kernel][block][wave][8] (slots 0..5 phases, 6 = steps, 7 = whole kernel).
__device__ unsigned long long* g_mlg_lstamps = nullptr;
struct LStamps {
    unsigned long long acc[6], last, begin, steps;
    __device__ void init() {
        for (int k = 0; k < 6; ++k) acc[k] = 0;
        steps = 0;
        last = begin = __builtin_amdgcn_s_memtime();
    }
    __device__ void mark(int k) {
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        acc[k] += now - last;
        last = now;
        __builtin_amdgcn_sched_barrier(0);
    }
    __device__ void flush(int kid) {
        if ((threadIdx.x & 63) || !g_mlg_lstamps) return;
        unsigned long long* o = g_mlg_lstamps + (((int64_t)kid * 1024 + blockIdx.x) * 8 + (threadIdx.x >> 6)) * 8;
        for (int k = 0; k < 6; ++k) o[k] = acc[k];
        o[6] = steps;
        o[7] = __builtin_amdgcn_s_memtime() - begin;
    }
};
#else
struct LStamps {
    unsigned long long steps;
    __device__ void init() {}
    __device__ void mark(int) {}
    __device__ void flush(int) {}
};
#endif
__device__ __forceinline__ int t_eff(const float* msum) { return (int)msum[1]; }


// ================================================================================================
// 16-row x 16-feature tile product with the activation operand in LDS, row-major [16][lda]:
// acc += W[m0 + col][kc*16 .. ] . act[row][kc*16 ..] over kchunks chunks.
__device__ __forceinline__ floatx4 tile_mm_lds(const float* __restrict__ W, int64_t ldw, int m0, const float* act, int lda,
                                               int kchunks, floatx4 acc, int lane) {
    const int col = lane & 15, g = lane >> 4;
    const float* wrow = W + (int64_t)(m0 + col) * ldw + 4 * g;
    const float* arow = act + col * lda + 4 * g;
    for (int kc = 0; kc < kchunks; ++kc) acc = mfma_chunk(ld4(wrow + kc * 16), ld4(arow + kc * 16), acc);
    return acc;
}


// ================================================================================================
// forward, split into the parallel (non-recurrent) and the recurrent part:
//   agent_in_kernel  (t, tile, net): dense input row (online), x = relu(fc1(inputs)), and
//                    GI = [b_ir + b_hr + W_ir x | b_iz + b_hz + W_iz x | b_in + W_in x]  for every timestep
//   agent_rec_kernel (tile, net):    h_t = GRU(GI_t, h_{t-1}) with W_hh in VGPRs, GI prefetched a step ahead
//   agent_q_kernel   (t, tile, net): q = fc2(h_t)
// The accumulation order per output is the one of the fused unroll (bias, W_ih x chunks, W_hh h chunks).
// grid (ntiles, T, 2), HC waves: wave w computes x chunk w, then GI chunks w, w + HC, w + 2 HC.
template <int H>
__global__ void __launch_bounds__(512) agent_in_kernel(LCfg c, MlgBatch bt, AgentLayout L, const float* __restrict__ Pon,
                                                       const float* __restrict__ Ptg, float* __restrict__ ws_in,
                                                       float* __restrict__ ws_x, float* __restrict__ gi_on,
                                                       float* __restrict__ gi_tg, const float* __restrict__ msum) {
    constexpr int HC = H / 16;
    constexpr int LDA = H + 4;
    __shared__ __attribute__((aligned(16))) float xs[16 * LDA];
    const int tile = blockIdx.x, t = blockIdx.y;
    if (t >= t_eff(msum)) return;
    const bool online = blockIdx.z == 0;
    const float* P = online ? Pon : Ptg;
    float* gi = online ? gi_on : gi_tg;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int col = lane & 15, g = lane >> 4;
    const int N = c.N, A = c.A, R = c.R;
    const int r = tile * 16 + col;
    const bool valid = r < R;
    const int b = valid ? r / N : 0, n = valid ? r % N : 0;
    const int64_t boff = (bslot(bt, b) * bt.T1 + t) * N + n;
    {
        floatx4 acc = ld4(P + L.b1 + w * 16 + 4 * g);
        if (valid) {
            if (L.last_action && t > 0) {
                // the one-hot row's only possible nonzero is at the recorded action (actions_onehot = OneHot(actions),
                // zero rows past an episode's end): one load of that element instead of a scan of the A columns
                const int a = (int)bt.actions[boff - N];
                const float v = (a >= 0 && a < A) ? bt.actions_onehot[(boff - N) * A + a] : 0.f;
                if (v != 0.f) acc += v * ld4(P + L.w1a + (int64_t)a * H + w * 16 + 4 * g);
            }
            if (L.agent_id) acc += ld4(P + L.w1n + (int64_t)n * H + w * 16 + 4 * g);
        }
        const float* orow = valid ? bt.obs + boff * c.d_obs : nullptr;
        const float* wrow = P + L.w1o + (int64_t)(w * 16 + col) * L.Dob + 4 * g;
        for (int kc = 0; kc < L.Dob / 16; ++kc)
            acc = mfma_chunk(ld4(wrow + kc * 16), load_chunk(orow, kc * 16 + 4 * g, c.d_obs), acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = fmaxf(acc[q], 0.f);
        *reinterpret_cast<floatx4*>(xs + col * LDA + w * 16 + 4 * g) = acc;
        if (online && valid) *reinterpret_cast<floatx4*>(ws_x + ((int64_t)t * R + r) * H + w * 16 + 4 * g) = acc;
    }
    if (online) {  // dense input row for dW1 (basic_controller.py:80-92 layout): 16 threads per row, one division per row
        const int l = tid & 15, oa = c.d_obs + (L.last_action ? A : 0);
        for (int i = tid >> 4; i < 16; i += blockDim.x >> 4) {
            const int rr = tile * 16 + i;
            if (rr >= R) break;
            const int bb = rr / N, nn = rr - bb * N;
            const int64_t bo = (bslot(bt, bb) * bt.T1 + t) * N + nn;
            float* dst = ws_in + ((int64_t)t * R + rr) * c.d_in;
            const float* src = bt.obs + bo * c.d_obs;
            for (int k = l; k < c.d_obs; k += 16) dst[k] = src[k];
            if (L.last_action)
                for (int k = l; k < A; k += 16) dst[c.d_obs + k] = t > 0 ? bt.actions_onehot[(bo - N) * A + k] : 0.f;
            for (int k = l; k < c.d_in - oa; k += 16) dst[oa + k] = k == nn ? 1.f : 0.f;
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; ++q) {  // gate q, feature chunk w
        floatx4 acc = q < 2 ? ld4(P + L.brz + q * H + w * 16 + 4 * g) : ld4(P + L.bih + 2 * H + w * 16 + 4 * g);
        acc = tile_mm_lds(P + L.wih, H, q * H + w * 16, xs, LDA, HC, acc, lane);
        if (valid) *reinterpret_cast<floatx4*>(gi + ((int64_t)t * R + r) * 3 * H + q * H + w * 16 + 4 * g) = acc;
    }
}

// grid (2 * ntiles): blockIdx < ntiles online (saves gates), else target. HC waves, wave w owns chunk w.
template <int H>
__global__ void __launch_bounds__(512) agent_rec_kernel(LCfg c, AgentLayout L, const float* __restrict__ Pon,
                                                        const float* __restrict__ Ptg, const float* __restrict__ gi_on,
                                                        const float* __restrict__ gi_tg, float* __restrict__ hs_on,
                                                        float* __restrict__ hs_tg, float* __restrict__ ws_gr,
                                                        float* __restrict__ ws_gz, float* __restrict__ ws_gn,
                                                        float* __restrict__ ws_ghn, const float* __restrict__ msum) {
    constexpr int HC = H / 16;
    constexpr int LDA = H + 4;
    __shared__ __attribute__((aligned(16))) float hs[2][16 * LDA];
    const int Te = t_eff(msum);
    const int ntiles = (c.R + 15) / 16;
    const bool online = blockIdx.x < ntiles;
    const int tile = online ? blockIdx.x : blockIdx.x - ntiles;
    const float* P = online ? Pon : Ptg;
    const float* gi = online ? gi_on : gi_tg;
    float* hsg = online ? hs_on : hs_tg;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int col = lane & 15, g = lane >> 4;
    const int R = c.R;
    const int r = tile * 16 + col;
    const bool valid = r < R;
    const int f0 = w * 16 + 4 * g;  // this lane's 4 hidden features
    floatx4 wr[3][HC];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int kc = 0; kc < HC; ++kc) wr[q][kc] = ld4(P + L.whh + (int64_t)(q * H + w * 16 + col) * H + kc * 16 + 4 * g);
    const floatx4 bhn = ld4(P + L.bhh + 2 * H + f0);
    for (int i = tid; i < 16 * LDA; i += blockDim.x) hs[0][i] = 0.f;
    if (valid) *reinterpret_cast<floatx4*>(hsg + (int64_t)r * H + f0) = floatx4{0.f, 0.f, 0.f, 0.f};  // HS[0]
    const int rr = valid ? r : 0;
    auto gi_at = [&](int t, int q) { return ld4(gi + ((int64_t)t * R + rr) * 3 * H + q * H + f0); };
    // input gates prefetched a step ahead into ping-pong registers: the 2x-unrolled loop consumes them in place,
    // so the wait for the prefetch never covers this step's stores (a register copy would force vmcnt(0))
    const __amdgpu_buffer_rsrc_t rs_h = mlg_rsrc(hsg), rs_r = mlg_rsrc(ws_gr), rs_z = mlg_rsrc(ws_gz),
                                 rs_n = mlg_rsrc(ws_gn), rs_hn = mlg_rsrc(ws_ghn);
    auto step = [&](int t, const floatx4 (&gc)[3], floatx4 (&gn)[3], int cur) {
        const int tn = t + 1 < Te ? t + 1 : t;  // unconditional (clamped) prefetch: no branch in the VMEM stream
#pragma unroll
        for (int q = 0; q < 3; ++q) gn[q] = gi_at(tn, q);
        floatx4 ar = gc[0], az = gc[1];
        floatx4 ahn = bhn;
        const float* hrow = hs[cur] + col * LDA + 4 * g;
#pragma unroll
        for (int kc = 0; kc < HC; ++kc) {
            const floatx4 hin = ld4(hrow + kc * 16);
            ar = mfma_chunk(wr[0][kc], hin, ar);
            az = mfma_chunk(wr[1][kc], hin, az);
            ahn = mfma_chunk(wr[2][kc], hin, ahn);
        }
        const floatx4 hp = ld4(hs[cur] + col * LDA + f0);
        floatx4 rg, zg, ng, hn;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            rg[q] = fast_sigmoid(ar[q]);
            zg[q] = fast_sigmoid(az[q]);
            ng[q] = fast_tanh(gc[2][q] + rg[q] * ahn[q]);
            hn[q] = ng[q] + zg[q] * (hp[q] - ng[q]);
        }
        *reinterpret_cast<floatx4*>(hs[cur ^ 1] + col * LDA + f0) = hn;
        const int64_t o = ((int64_t)t * R + r) * H + f0;
        st4_if(rs_h, o + (int64_t)R * H, hn, valid);  // HS[t + 1]
        st4_if(rs_r, o, rg, valid && online);          // gates are saved by the online net only
        st4_if(rs_z, o, zg, valid && online);
        st4_if(rs_n, o, ng, valid && online);
        st4_if(rs_hn, o, ahn, valid && online);
        __syncthreads();
    };
    floatx4 ga[3], gb[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) ga[q] = gi_at(0, q);
    __syncthreads();
    // step 0 peeled: the loop is entered in the same VMEM state as its back edge (prefetch loads, then the
    // stores), so the compiler's merged waitcnt for the prefetched gates still lets the stores drain
    step(0, ga, gb, 0);
    for (int t = 1; t < Te; t += 2) {
        step(t, gb, ga, 1);
        if (t + 1 < Te) step(t + 1, ga, gb, 0);
    }
}

// The recurrence on 4-row tiles with v_mfma_f32_4x4x1_16b_f32 (16 blocks of D[4x4] += A[4x1] B[1x4]; lane
// 4b + i supplies A_b[i], lane 4b + j supplies B_b[j], D_b[i][j] is register i of lane 4b + j). A 16-row tile
// per CU is MFMA-bound at 48 16x16x4 MFMAs per SIMD per step; 4-row tiles put 4x as many CUs on the
// sequential T loop. Wave w owns hidden features 16w..16w+15: block b = 4g + fg computes gate g (r, z, W_hn h;
// g = 3 idle) of features 16w + 4fg + i for the tile's 4 rows, W_hh rows of the block in VGPRs (H per lane).
// A row / register transpose across the wave's four 16-lane rows (rows_transpose4, four VALU lane swaps) then
// gives every lane the three gates of one (feature 16w + 4fg + g, row): all 64 lanes finish one GRU cell each.
// grid (2 * ntiles4): blockIdx < ntiles4 online (saves gates), else target. H/16 waves.
template <int H>
__device__ __forceinline__ void agent_rec4_body(const LCfg& c, const AgentLayout& L, const float* __restrict__ Pon,
                                                const float* __restrict__ Ptg, const float* __restrict__ gi_on,
                                                const float* __restrict__ gi_tg, float* __restrict__ hs_on,
                                                float* __restrict__ hs_tg, float* __restrict__ ws_gr,
                                                float* __restrict__ ws_gz, float* __restrict__ ws_gn,
                                                float* __restrict__ ws_ghn, const float* __restrict__ msum, int bid) {
    LStamps lst;
    lst.init();
    const int nt4 = (c.R + 3) / 4;
    const bool online = bid < nt4;
    const float* P = online ? Pon : Ptg;
    const mlg::Gru4Fwd a{c.R, P + L.whh, P + L.bhh, online ? gi_on : gi_tg, online ? hs_on : hs_tg,
                         ws_gr, ws_gz, ws_gn, ws_ghn, online};
    mlg::gru4_fwd<H>(a, online ? bid : bid - nt4, t_eff(msum), lst);
    lst.flush(0);
}

template <int H>
__global__ void __launch_bounds__(512) agent_rec4_kernel(LCfg c, AgentLayout L, const float* __restrict__ Pon,
                                                         const float* __restrict__ Ptg, const float* __restrict__ gi_on,
                                                         const float* __restrict__ gi_tg, float* __restrict__ hs_on,
                                                         float* __restrict__ hs_tg, float* __restrict__ ws_gr,
                                                         float* __restrict__ ws_gz, float* __restrict__ ws_gn,
                                                         float* __restrict__ ws_ghn, const float* __restrict__ msum) {
    agent_rec4_body<H>(c, L, Pon, Ptg, gi_on, gi_tg, hs_on, hs_tg, ws_gr, ws_gz, ws_gn, ws_ghn, msum, blockIdx.x);
}

// grid (ntiles, T, 2), Ap/16 waves: wave = action tile. q = b2 + W2 . h_t (h_t = HS[t + 1]).
template <int H>
__global__ void __launch_bounds__(512) agent_q_kernel(LCfg c, AgentLayout L, const float* __restrict__ Pon,
                                                      const float* __restrict__ Ptg, const float* __restrict__ hs_on,
                                                      const float* __restrict__ hs_tg, float* __restrict__ mac,
                                                      float* __restrict__ tmac, const float* __restrict__ msum) {
    constexpr int HC = H / 16;
    const int tile = blockIdx.x, t = blockIdx.y;
    if (t >= t_eff(msum)) return;
    const bool online = blockIdx.z == 0;
    const float* P = online ? Pon : Ptg;
    const float* hsg = (online ? hs_on : hs_tg) + (int64_t)(t + 1) * c.R * H;
    float* qout = online ? mac : tmac;
    const int lane = threadIdx.x & 63, at = threadIdx.x >> 6;
    const int col = lane & 15, g = lane >> 4;
    const int r = tile * 16 + col;
    const bool valid = r < c.R;
    const float* hrow = hsg + (int64_t)(valid ? r : 0) * H + 4 * g;
    const float* wrow = P + L.w2 + (int64_t)(at * 16 + col) * H + 4 * g;
    floatx4 q = ld4(P + L.b2 + at * 16 + 4 * g);
#pragma unroll
    for (int kc = 0; kc < HC; ++kc) q = mfma_chunk(ld4(wrow + kc * 16), ld4(hrow + kc * 16), q);
    if (valid) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int a = at * 16 + 4 * g + k;
            if (a < c.A) qout[((int64_t)t * c.R + r) * c.A + a] = q[k];
        }
    }
}

// ================================================================================================
// QMixer on one 16-row tile (rows on lanes).  l1 = [w1h | wfh | b1 | vh] (post ReLU except b1).
template <int HE, int E>
struct Mixer {
    static constexpr int T1H = HE / 16, TE = E / 16, L1T = (2 * HE + 2 * E) / 16;
    static constexpr int OW1 = 0, OWF = T1H, OB1 = 2 * T1H, OVH = 2 * T1H + TE;

    // first layer + ReLUs; s = this lane's state row (nullptr -> zeros)
    __device__ static void layer1(const MixPtrs& M, const MixPack& mp, int S, const float* s, floatx4 (&l1)[L1T], int lane) {
        const int col = lane & 15, g = lane >> 4;
#pragma unroll
        for (int mt = 0; mt < L1T; ++mt) l1[mt] = ld4(M.mb1 + mt * 16 + 4 * g);
        for (int kc = 0; kc < mp.Sp / 16; ++kc) {
            const floatx4 sv = load_chunk(s, kc * 16 + 4 * g, S);
#pragma unroll
            for (int mt = 0; mt < L1T; ++mt)
                l1[mt] = mfma_chunk(ld4(M.m1 + (int64_t)(mt * 16 + col) * mp.Sp + kc * 16 + 4 * g), sv, l1[mt]);
        }
#pragma unroll
        for (int mt = 0; mt < L1T; ++mt) {
            if (mt >= OB1 && mt < OVH) continue;
#pragma unroll
            for (int q = 0; q < 4; ++q) l1[mt][q] = fmaxf(l1[mt][q], 0.f);
        }
    }

    // pre-abs hyper_w_1 output for agent n, chunk cc (features n*E + cc*16 ..)
    __device__ static floatx4 w1pre(const MixPtrs& M, int n, int cc, const floatx4 (&l1)[L1T], int lane) {
        const int col = lane & 15, g = lane >> 4;
        floatx4 acc = ld4(M.ba2 + n * E + cc * 16 + 4 * g);
        const float* wrow = M.a2 + (int64_t)(n * E + cc * 16 + col) * HE + 4 * g;
#pragma unroll
        for (int kc = 0; kc < T1H; ++kc) acc = mfma_chunk(ld4(wrow + kc * 16), l1[OW1 + kc], acc);
        return acc;
    }

    __device__ static floatx4 wfpre(const MixPtrs& M, int cc, const floatx4 (&l1)[L1T], int lane) {
        const int col = lane & 15, g = lane >> 4;
        floatx4 acc = ld4(M.bf2 + cc * 16 + 4 * g);
        const float* wrow = M.f2 + (int64_t)(cc * 16 + col) * HE + 4 * g;
#pragma unroll
        for (int kc = 0; kc < T1H; ++kc) acc = mfma_chunk(ld4(wrow + kc * 16), l1[OWF + kc], acc);
        return acc;
    }

    __device__ static float vval(const MixPtrs& M, const floatx4 (&l1)[L1T], int lane) {
        const int col = lane & 15, g = lane >> 4;
        floatx4 acc = ld4(M.bv2p + 4 * g);
        const float* wrow = M.v2p + (int64_t)col * E + 4 * g;
#pragma unroll
        for (int kc = 0; kc < TE; ++kc) acc = mfma_chunk(ld4(wrow + kc * 16), l1[OVH + kc], acc);
        return __shfl(acc[0], col);  // feature 0 lives in lane group 0, reg 0
    }

    // forward: y per row (identical in the 4 lanes of a row). q(n) = this row's agent-n value.
    __device__ static float forward(const MixPtrs& M, const MixPack& mp, int S, int N, const float* s, const float* qrow,
                                    floatx4 (&l1)[L1T], floatx4 (&pre)[TE], floatx4 (&hid)[TE], floatx4 (&wfp)[TE], int lane) {
        layer1(M, mp, S, s, l1, lane);
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) pre[cc] = l1[OB1 + cc];
        for (int n = 0; n < N; ++n) {
            const float qn = qrow[n];
#pragma unroll
            for (int cc = 0; cc < TE; ++cc) {
                const floatx4 wp = w1pre(M, n, cc, l1, lane);
#pragma unroll
                for (int q = 0; q < 4; ++q) pre[cc][q] += qn * fabsf(wp[q]);
            }
        }
        float part = 0.f;
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) {
            wfp[cc] = wfpre(M, cc, l1, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                hid[cc][q] = pre[cc][q] > 0.f ? pre[cc][q] : expm1f(pre[cc][q]);
                part += hid[cc][q] * fabsf(wfp[cc][q]);
            }
        }
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
        return part + vval(M, l1, lane);
    }
};

// The same QMixer forward with every weight operand of a stage loaded up front (one L2 round trip per stage
// instead of one per 16-wide K chunk: the mix_td waves are L2-latency-bound, one wave per SIMD, so registers are
// plentiful). State rows of at most SPC * 16 features, at most NMAX agents; identical arithmetic to Mixer. w1p
// keeps the pre-abs hyper_w_1 outputs for the backward.
template <int HE, int E, int SPC, int NMAX>
struct MixerPF {
    using Mx = Mixer<HE, E>;
    static constexpr int T1H = Mx::T1H, TE = Mx::TE, L1T = Mx::L1T;
    static constexpr int OW1 = Mx::OW1, OWF = Mx::OWF, OB1 = Mx::OB1, OVH = Mx::OVH;

    // The state-only half of forward(): layer 1, hyper_w_1's second layer for every agent (pre-abs), hyper_w_final's
    // second layer (pre-abs) and V(s) (identical in the 4 lanes of a row). Same operations as forward().
    __device__ static void hyper(const MixPtrs& M, const MixPack& mp, int S, int N, const float* s, floatx4 (&l1)[L1T],
                                 floatx4 (&w1p)[NMAX][TE], floatx4 (&wfp)[TE], float& v, int lane) {
        const int col = lane & 15, g = lane >> 4;
        {  // layer 1
            floatx4 sv[SPC], wl[L1T][SPC];
#pragma unroll
            for (int kc = 0; kc < SPC; ++kc) sv[kc] = load_chunk(s, kc * 16 + 4 * g, S);
#pragma unroll
            for (int mt = 0; mt < L1T; ++mt) {
                l1[mt] = ld4(M.mb1 + mt * 16 + 4 * g);
#pragma unroll
                for (int kc = 0; kc < SPC; ++kc) wl[mt][kc] = ld4(M.m1 + (int64_t)(mt * 16 + col) * mp.Sp + kc * 16 + 4 * g);
            }
#pragma unroll
            for (int kc = 0; kc < SPC; ++kc)
#pragma unroll
                for (int mt = 0; mt < L1T; ++mt) l1[mt] = mfma_chunk(wl[mt][kc], sv[kc], l1[mt]);
#pragma unroll
            for (int mt = 0; mt < L1T; ++mt) {
                if (mt >= OB1 && mt < OVH) continue;
#pragma unroll
                for (int q = 0; q < 4; ++q) l1[mt][q] = fmaxf(l1[mt][q], 0.f);
            }
        }
#pragma unroll
        for (int n = 0; n < NMAX; ++n) {
            if (n >= N) break;
            floatx4 wa[TE][T1H];
#pragma unroll
            for (int cc = 0; cc < TE; ++cc) {
                w1p[n][cc] = ld4(M.ba2 + n * E + cc * 16 + 4 * g);
#pragma unroll
                for (int kc = 0; kc < T1H; ++kc)
                    wa[cc][kc] = ld4(M.a2 + (int64_t)(n * E + cc * 16 + col) * HE + kc * 16 + 4 * g);
            }
#pragma unroll
            for (int cc = 0; cc < TE; ++cc)
#pragma unroll
                for (int kc = 0; kc < T1H; ++kc) w1p[n][cc] = mfma_chunk(wa[cc][kc], l1[OW1 + kc], w1p[n][cc]);
        }
        floatx4 wf[TE][T1H], wv[TE];
        floatx4 bv = ld4(M.bv2p + 4 * g);
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) {
            wfp[cc] = ld4(M.bf2 + cc * 16 + 4 * g);
            wv[cc] = ld4(M.v2p + (int64_t)col * E + cc * 16 + 4 * g);
#pragma unroll
            for (int kc = 0; kc < T1H; ++kc) wf[cc][kc] = ld4(M.f2 + (int64_t)(cc * 16 + col) * HE + kc * 16 + 4 * g);
        }
#pragma unroll
        for (int cc = 0; cc < TE; ++cc)
#pragma unroll
            for (int kc = 0; kc < T1H; ++kc) wfp[cc] = mfma_chunk(wf[cc][kc], l1[OWF + kc], wfp[cc]);
#pragma unroll
        for (int kc = 0; kc < TE; ++kc) bv = mfma_chunk(wv[kc], l1[OVH + kc], bv);
        v = __shfl(bv[0], col);
    }

    // The Q-dependent half: the mixing with hyper()'s outputs (b1 = layer-1 tiles OB1..), forward()'s order.
    __device__ static float mix(int N, const float* qrow, const floatx4 (&b1)[TE], const floatx4 (&w1p)[NMAX][TE],
                                const floatx4 (&wfp)[TE], float v, floatx4 (&pre)[TE], floatx4 (&hid)[TE]) {
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) pre[cc] = b1[cc];
#pragma unroll
        for (int n = 0; n < NMAX; ++n) {
            if (n >= N) break;
            const float qn = qrow[n];
#pragma unroll
            for (int cc = 0; cc < TE; ++cc)
#pragma unroll
                for (int q = 0; q < 4; ++q) pre[cc][q] += qn * fabsf(w1p[n][cc][q]);
        }
        float part = 0.f;
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                hid[cc][q] = pre[cc][q] > 0.f ? pre[cc][q] : expm1f(pre[cc][q]);
                part += hid[cc][q] * fabsf(wfp[cc][q]);
            }
        }
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
        return part + v;
    }

    __device__ static float forward(const MixPtrs& M, const MixPack& mp, int S, int N, const float* s, const float* qrow,
                                    floatx4 (&l1)[L1T], floatx4 (&pre)[TE], floatx4 (&hid)[TE], floatx4 (&wfp)[TE],
                                    floatx4 (&w1p)[NMAX][TE], int lane) {
        const int col = lane & 15, g = lane >> 4;
        {  // layer 1
            floatx4 sv[SPC], wl[L1T][SPC];
#pragma unroll
            for (int kc = 0; kc < SPC; ++kc) sv[kc] = load_chunk(s, kc * 16 + 4 * g, S);
#pragma unroll
            for (int mt = 0; mt < L1T; ++mt) {
                l1[mt] = ld4(M.mb1 + mt * 16 + 4 * g);
#pragma unroll
                for (int kc = 0; kc < SPC; ++kc) wl[mt][kc] = ld4(M.m1 + (int64_t)(mt * 16 + col) * mp.Sp + kc * 16 + 4 * g);
            }
#pragma unroll
            for (int kc = 0; kc < SPC; ++kc)
#pragma unroll
                for (int mt = 0; mt < L1T; ++mt) l1[mt] = mfma_chunk(wl[mt][kc], sv[kc], l1[mt]);
#pragma unroll
            for (int mt = 0; mt < L1T; ++mt) {
                if (mt >= OB1 && mt < OVH) continue;
#pragma unroll
                for (int q = 0; q < 4; ++q) l1[mt][q] = fmaxf(l1[mt][q], 0.f);
            }
        }
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) pre[cc] = l1[OB1 + cc];
#pragma unroll
        for (int n = 0; n < NMAX; ++n) {  // hyper_w_1 second layer for every agent: weights of all agents first
            if (n >= N) break;
            floatx4 wa[TE][T1H];
#pragma unroll
            for (int cc = 0; cc < TE; ++cc) {
                w1p[n][cc] = ld4(M.ba2 + n * E + cc * 16 + 4 * g);
#pragma unroll
                for (int kc = 0; kc < T1H; ++kc)
                    wa[cc][kc] = ld4(M.a2 + (int64_t)(n * E + cc * 16 + col) * HE + kc * 16 + 4 * g);
            }
#pragma unroll
            for (int cc = 0; cc < TE; ++cc)
#pragma unroll
                for (int kc = 0; kc < T1H; ++kc) w1p[n][cc] = mfma_chunk(wa[cc][kc], l1[OW1 + kc], w1p[n][cc]);
        }
#pragma unroll
        for (int n = 0; n < NMAX; ++n) {
            if (n >= N) break;
            const float qn = qrow[n];
#pragma unroll
            for (int cc = 0; cc < TE; ++cc)
#pragma unroll
                for (int q = 0; q < 4; ++q) pre[cc][q] += qn * fabsf(w1p[n][cc][q]);
        }
        floatx4 wf[TE][T1H], wv[TE];
        floatx4 bv = ld4(M.bv2p + 4 * g);
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) {
            wfp[cc] = ld4(M.bf2 + cc * 16 + 4 * g);
            wv[cc] = ld4(M.v2p + (int64_t)col * E + cc * 16 + 4 * g);
#pragma unroll
            for (int kc = 0; kc < T1H; ++kc) wf[cc][kc] = ld4(M.f2 + (int64_t)(cc * 16 + col) * HE + kc * 16 + 4 * g);
        }
        float part = 0.f;
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) {
#pragma unroll
            for (int kc = 0; kc < T1H; ++kc) wfp[cc] = mfma_chunk(wf[cc][kc], l1[OWF + kc], wfp[cc]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                hid[cc][q] = pre[cc][q] > 0.f ? pre[cc][q] : expm1f(pre[cc][q]);
                part += hid[cc][q] * fabsf(wfp[cc][q]);
            }
        }
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
#pragma unroll
        for (int kc = 0; kc < TE; ++kc) bv = mfma_chunk(wv[kc], l1[OVH + kc], bv);
        return part + __shfl(bv[0], col);
    }
};

__device__ __forceinline__ float row_sum16(float v) {  // sum over the 16 lanes of lane group 0
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    return v;
}

// chosen / target per-agent values of row (b, t) (q_learner.py:55, 68-75)
__device__ __forceinline__ void gather_q(const LCfg& c, const MlgBatch& bt, const float* mac, const float* tmac, int b, int t,
                                         float* cq, float* tq) {
    const int N = c.N, A = c.A, R = c.R;
    for (int n = 0; n < N; ++n) {
        const int r = b * N + n;
        const int a = (int)bt.actions[(bslot(bt, b) * bt.T1 + t) * N + n];
        cq[n] = mac[((int64_t)t * R + r) * A + a];
        const int32_t* av = bt.avail + (bslot(bt, b) * bt.T1 + t + 1) * N * A + (int64_t)n * A;
        const float* qn = mac + ((int64_t)(t + 1) * R + r) * A;
        const float* tn = tmac + ((int64_t)(t + 1) * R + r) * A;
        if (c.double_q) {
            float bv = 0.f;
            int bi = 0;
            for (int k = 0; k < A; ++k) {
                const float v = av[k] ? qn[k] : -9999999.f;
                if (k == 0 || v > bv) { bv = v; bi = k; }
            }
            tq[n] = av[bi] ? tn[bi] : -9999999.f;
        } else {
            float bv = 0.f;
            for (int k = 0; k < A; ++k) {
                const float v = av[k] ? tn[k] : -9999999.f;
                if (k == 0 || v > bv) bv = v;
            }
            tq[n] = bv;
        }
    }
}

constexpr int MIXPF_N = 8, MIXPF_A = 16;  // mix_td FAST path bounds (agents, actions)

// gather_q with every load of an agent issued together (A <= AMAX): avail row, online next-step Q, target
// next-step Q; same selection rule and order as gather_q.
template <int AMAX>
__device__ __forceinline__ void gather_q_pf(const LCfg& c, const MlgBatch& bt, const float* mac, const float* tmac, int b,
                                            int t, float* cq, float* tq) {
    const int N = c.N, A = c.A, R = c.R;
    const int64_t row0 = (bslot(bt, b) * bt.T1 + t) * N;
#pragma unroll
    for (int n = 0; n < MIXPF_N; ++n) {  // unrolled: cq / tq stay in registers
        if (n >= N) break;
        const int r = b * N + n;
        const int a = (int)bt.actions[row0 + n];
        const int32_t* av = bt.avail + (bslot(bt, b) * bt.T1 + t + 1) * N * A + (int64_t)n * A;
        const float* qn = mac + ((int64_t)(t + 1) * R + r) * A;
        const float* tn = tmac + ((int64_t)(t + 1) * R + r) * A;
        int avv[AMAX];
        float qv[AMAX], tv[AMAX];
#pragma unroll
        for (int k = 0; k < AMAX; ++k) {
            const bool in = k < A;
            avv[k] = in ? av[k] : 0;
            qv[k] = in ? qn[k] : 0.f;
            tv[k] = in ? tn[k] : 0.f;
        }
        cq[n] = mac[((int64_t)t * R + r) * A + a];
        if (c.double_q) {
            float bv = 0.f;
            int bi = 0;
#pragma unroll
            for (int k = 0; k < AMAX; ++k) {
                if (k >= A) break;
                const float v = avv[k] ? qv[k] : -9999999.f;
                const bool take = k == 0 || v > bv;
                bv = take ? v : bv;
                bi = take ? k : bi;
            }
            float tb = 0.f;
            int ab = 0;
#pragma unroll
            for (int k = 0; k < AMAX; ++k) {  // tv[bi], avv[bi] without dynamic register indexing
                tb = k == bi ? tv[k] : tb;
                ab = k == bi ? avv[k] : ab;
            }
            tq[n] = ab ? tb : -9999999.f;
        } else {
            float bv = 0.f;
#pragma unroll
            for (int k = 0; k < AMAX; ++k) {
                if (k >= A) break;
                const float v = avv[k] ? tv[k] : -9999999.f;
                bv = (k == 0 || v > bv) ? v : bv;
            }
            tq[n] = bv;
        }
    }
}

constexpr int MAXN = 32;

// gather_q_pf with the agents spread over the four 16-lane rows (row g takes agents g, g + 4, ...: the rows of a D
// layout hold the same (b, t) row, so gather_q_pf loaded everything four times) and the values all-gathered back by
// rows_transpose4 (VALU lane swaps). Same selection rule per agent; N <= 8.
template <int AMAX>
__device__ __forceinline__ void gather_q_rows(const LCfg& c, const MlgBatch& bt, const float* mac, const float* tmac, int b,
                                              int t, bool valid, int g, float* cq, float* tq) {
    const int N = c.N, A = c.A, R = c.R;
    const int64_t row0 = (bslot(bt, b) * bt.T1 + t) * N;
    float cv[2], tv[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int n = g + 4 * i;
        cv[i] = tv[i] = 0.f;
        if (!valid || n >= N) continue;
        const int r = b * N + n;
        const int a = (int)bt.actions[row0 + n];
        const int32_t* av = bt.avail + (bslot(bt, b) * bt.T1 + t + 1) * N * A + (int64_t)n * A;
        const float* qn = mac + ((int64_t)(t + 1) * R + r) * A;
        const float* tn = tmac + ((int64_t)(t + 1) * R + r) * A;
        int avv[AMAX];
        float qv[AMAX], tvv[AMAX];
#pragma unroll
        for (int k = 0; k < AMAX; ++k) {
            const bool in = k < A;
            avv[k] = in ? av[k] : 0;
            qv[k] = in ? qn[k] : 0.f;
            tvv[k] = in ? tn[k] : 0.f;
        }
        cv[i] = mac[((int64_t)t * R + r) * A + a];
        if (c.double_q) {
            float bv = 0.f;
            int bi = 0;
#pragma unroll
            for (int k = 0; k < AMAX; ++k) {
                if (k >= A) break;
                const float v = avv[k] ? qv[k] : -9999999.f;
                const bool take = k == 0 || v > bv;
                bv = take ? v : bv;
                bi = take ? k : bi;
            }
            float tb = 0.f;
            int ab = 0;
#pragma unroll
            for (int k = 0; k < AMAX; ++k) {
                tb = k == bi ? tvv[k] : tb;
                ab = k == bi ? avv[k] : ab;
            }
            tv[i] = ab ? tb : -9999999.f;
        } else {
            float bv = 0.f;
#pragma unroll
            for (int k = 0; k < AMAX; ++k) {
                if (k >= A) break;
                const float v = avv[k] ? tvv[k] : -9999999.f;
                bv = (k == 0 || v > bv) ? v : bv;
            }
            tv[i] = bv;
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // row p's value of agent p + 4 i to every row
        float c0 = cv[i], c1 = cv[i], c2 = cv[i], c3 = cv[i];
        float t0 = tv[i], t1 = tv[i], t2 = tv[i], t3 = tv[i];
        rows_transpose4(c0, c1, c2, c3);
        rows_transpose4(t0, t1, t2, t3);
        const float cs[4] = {c0, c1, c2, c3}, ts[4] = {t0, t1, t2, t3};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if (4 * i + p >= MIXPF_N) break;
            cq[4 * i + p] = cs[p];
            tq[4 * i + p] = ts[p];
        }
    }
}

struct MixOut {
    float *srow, *l1act, *d1, *da2, *df2, *dv2, *dq, *d2, *part;
};

// FAST (state rows of <= 64 features, <= 8 agents, <= 16 actions): the prefetching mixer forward (MixerPF), the
// backward reusing its hyper_w_1 outputs with the W_a2^T / W_f2^T operands loaded up front, gather_q_pf.
// Identical arithmetic either way.
template <int HE, int E, bool FAST = false>
__global__ void __launch_bounds__(128) mix_td_kernel(LCfg c, MlgBatch bt, MixPtrs Mon, MixPtrs Mtg, MixPack mp,
                                                    const float* __restrict__ mac, const float* __restrict__ tmac,
                                                    const float* __restrict__ msum_p, MixOut o) {
    using Mx = Mixer<HE, E>;
    using MP = MixerPF<HE, E, 4, MIXPF_N>;
    floatx4 w1c[MIXPF_N][Mx::TE];  // FAST: the online forward's pre-abs hyper_w_1 outputs
    // two waves per 16-row tile: wave 0 runs the target mixer forward and hands y's target to wave 1 through LDS,
    // wave 1 runs the online forward, TD and the mixer backward (VDN: wave 1 alone)
    __shared__ float tgt_sh[16];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, col = lane & 15, g = lane >> 4;
    if (c.mixer != 2 && wv == 0) return;
    const int rm = blockIdx.x * 16 + col;
    const int Tm = c.T - 1;
    const bool valid = rm < c.RM;
    const int b = valid ? rm / Tm : 0, t = valid ? rm % Tm : 0;
    const int N = c.N, S = c.S, L1 = 2 * HE + 2 * E, NE = N * E;
    float cq[MAXN], tq[MAXN];
    for (int n = 0; n < N; ++n) cq[n] = tq[n] = 0.f;
    if (valid) {
        if constexpr (FAST)
            gather_q_pf<MIXPF_A>(c, bt, mac, tmac, b, t, cq, tq);
        else
            gather_q(c, bt, mac, tmac, b, t, cq, tq);
    }
    const float m = (valid && t < t_eff(msum_p) - 1) ? mask_at(bt, b, t) : 0.f;  // reference truncation
    const float rwd = valid ? bt.reward[bslot(bt, b) * bt.T1 + t] : 0.f;
    const float term = valid ? (float)bt.terminated[bslot(bt, b) * bt.T1 + t] : 0.f;
    const float msum = msum_p[0];
    const float* s0 = valid ? bt.state + (bslot(bt, b) * bt.T1 + t) * S : nullptr;
    const float* s1 = valid ? bt.state + (bslot(bt, b) * bt.T1 + t + 1) * S : nullptr;
    float qtot, tgt;
    floatx4 l1[Mx::L1T], pre[Mx::TE], hid[Mx::TE], wfp[Mx::TE];
    if (c.mixer == 2) {
        if (wv == 0) {
            floatx4 tl1[Mx::L1T], tpre[Mx::TE], thid[Mx::TE], twfp[Mx::TE];
            float tv;
            if constexpr (FAST) {
                floatx4 tw1c[MIXPF_N][Mx::TE];
                tv = MP::forward(Mtg, mp, S, N, s1, tq, tl1, tpre, thid, twfp, tw1c, lane);
            } else {
                tv = Mx::forward(Mtg, mp, S, N, s1, tq, tl1, tpre, thid, twfp, lane);
            }
            if (g == 0) tgt_sh[col] = tv;
            qtot = 0.f;
        } else {
            if constexpr (FAST)
                qtot = MP::forward(Mon, mp, S, N, s0, cq, l1, pre, hid, wfp, w1c, lane);
            else
                qtot = Mx::forward(Mon, mp, S, N, s0, cq, l1, pre, hid, wfp, lane);
        }
        __syncthreads();
        if (wv == 0) return;
        tgt = tgt_sh[col];
    } else {  // VDN (vdn.py:9)
        qtot = 0.f;
        tgt = 0.f;
        for (int n = 0; n < N; ++n) {
            qtot += cq[n];
            tgt += tq[n];
        }
    }
    const float y = rwd + c.gamma * (1.f - term) * tgt;          // q_learner.py:86
    const float mtd = (qtot - y) * m;                             // :89-95
    const float dy = 2.f * mtd * m / msum;                        // d loss / d q_tot
    // ---- loss / stat partials (one row per lane of group 0) ----
    {
        float p0 = g == 0 ? mtd * mtd : 0.f, p1 = g == 0 ? fabsf(mtd) : 0.f;
        float p2 = g == 0 ? qtot * m : 0.f, p3 = g == 0 ? y * m : 0.f;
        p0 = row_sum16(p0);
        p1 = row_sum16(p1);
        p2 = row_sum16(p2);
        p3 = row_sum16(p3);
        if (lane == 0) {
            float* pp = o.part + (int64_t)blockIdx.x * 4;
            pp[0] = p0;
            pp[1] = p1;
            pp[2] = p2;
            pp[3] = p3;
        }
    }
    float dq[MAXN];
    if (c.mixer == 2) {
        // ---- QMixer backward (autograd of qmix.py:41-59) ----
        floatx4 dpre[Mx::TE], dwf[Mx::TE];
#pragma unroll
        for (int cc = 0; cc < Mx::TE; ++cc) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float dh = dy * fabsf(wfp[cc][q]);
                const float sg = wfp[cc][q] > 0.f ? 1.f : (wfp[cc][q] < 0.f ? -1.f : 0.f);
                dwf[cc][q] = dy * hid[cc][q] * sg;
                dpre[cc][q] = pre[cc][q] > 0.f ? dh : dh * (hid[cc][q] + 1.f);
            }
        }
        floatx4 dw1h[Mx::T1H];
#pragma unroll
        for (int mt = 0; mt < Mx::T1H; ++mt) dw1h[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int n = 0; n < N; ++n) {
            float part = 0.f;
            floatx4 aT[Mx::TE][Mx::T1H];  // FAST: this agent's W_a2^T operands, loaded before its MFMAs
            if constexpr (FAST) {
#pragma unroll
                for (int cc = 0; cc < Mx::TE; ++cc)
#pragma unroll
                    for (int mt = 0; mt < Mx::T1H; ++mt)
                        aT[cc][mt] = ld4(Mon.a2T + (int64_t)(mt * 16 + col) * NE + n * E + cc * 16 + 4 * g);
            }
#pragma unroll
            for (int cc = 0; cc < Mx::TE; ++cc) {
                floatx4 wp;
                if constexpr (FAST) {
                    floatx4 wsel = w1c[0][cc];  // w1c[n][cc] without dynamic register indexing
#pragma unroll
                    for (int k = 1; k < MIXPF_N; ++k)
                        if (k == n) wsel = w1c[k][cc];
                    wp = wsel;
                } else {
                    wp = Mx::w1pre(Mon, n, cc, l1, lane);
                }
                floatx4 dlt;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    part += fabsf(wp[q]) * dpre[cc][q];
                    const float sg = wp[q] > 0.f ? 1.f : (wp[q] < 0.f ? -1.f : 0.f);
                    dlt[q] = cq[n] * dpre[cc][q] * sg;
                }
                if (valid) *reinterpret_cast<floatx4*>(o.da2 + (int64_t)rm * NE + n * E + cc * 16 + 4 * g) = dlt;
                // dw1h += W_a2^T[:, n*E + cc*16 ..] . dlt   (a2T is [HE][NE])
#pragma unroll
                for (int mt = 0; mt < Mx::T1H; ++mt) {
                    floatx4 wa;
                    if constexpr (FAST)
                        wa = aT[cc][mt];
                    else
                        wa = ld4(Mon.a2T + (int64_t)(mt * 16 + col) * NE + n * E + cc * 16 + 4 * g);
                    dw1h[mt] = mfma_chunk(wa, dlt, dw1h[mt]);
                }
            }
            part += __shfl_xor(part, 16);
            part += __shfl_xor(part, 32);
            dq[n] = part;
        }
        // dwfh = W_f2^T . dwf -- MFMA needs every lane active, so it runs outside the store guard
        floatx4 dwfh[Mx::T1H];
#pragma unroll
        for (int mt = 0; mt < Mx::T1H; ++mt) {
            floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int cc = 0; cc < Mx::TE; ++cc)
                acc = mfma_chunk(ld4(Mon.f2T + (int64_t)(mt * 16 + col) * E + cc * 16 + 4 * g), dwf[cc], acc);
            dwfh[mt] = acc;
        }
        if (valid) {
            float* d1 = o.d1 + (int64_t)rm * L1;
            float* la = o.l1act + (int64_t)rm * L1;
#pragma unroll
            for (int mt = 0; mt < Mx::T1H; ++mt) {  // w1h
                floatx4 v;
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = l1[Mx::OW1 + mt][q] > 0.f ? dw1h[mt][q] : 0.f;
                *reinterpret_cast<floatx4*>(d1 + mt * 16 + 4 * g) = v;
            }
#pragma unroll
            for (int mt = 0; mt < Mx::T1H; ++mt) {  // wfh
                floatx4 acc = dwfh[mt];
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[q] = l1[Mx::OWF + mt][q] > 0.f ? acc[q] : 0.f;
                *reinterpret_cast<floatx4*>(d1 + HE + mt * 16 + 4 * g) = acc;
            }
#pragma unroll
            for (int cc = 0; cc < Mx::TE; ++cc) {  // b1, vh
                *reinterpret_cast<floatx4*>(d1 + 2 * HE + cc * 16 + 4 * g) = dpre[cc];
                const floatx4 wv = ld4(Mon.v2p + cc * 16 + 4 * g);
                floatx4 v;
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = l1[Mx::OVH + cc][q] > 0.f ? dy * wv[q] : 0.f;
                *reinterpret_cast<floatx4*>(d1 + 2 * HE + E + cc * 16 + 4 * g) = v;
                *reinterpret_cast<floatx4*>(o.df2 + (int64_t)rm * E + cc * 16 + 4 * g) = dwf[cc];
            }
#pragma unroll
            for (int mt = 0; mt < Mx::L1T; ++mt) *reinterpret_cast<floatx4*>(la + mt * 16 + 4 * g) = l1[mt];
            if (g == 0) {
                o.dv2[rm] = dy;
                for (int k = 0; k < S; ++k) o.srow[(int64_t)rm * S + k] = s0[k];
            }
        }
    } else {
        for (int n = 0; n < N; ++n) dq[n] = dy;
    }
    // ---- dQ per agent row (t-major) and its one-hot expansion for dW2 ----
    if (valid && g == 0) {
        for (int n = 0; n < N; ++n) {
            const int r = b * N + n;
            o.dq[(int64_t)t * c.R + r] = dq[n];
            const int a = (int)bt.actions[(bslot(bt, b) * bt.T1 + t) * N + n];
            o.d2[((int64_t)t * c.R + r) * c.A + a] = dq[n];
        }
    }
}

// ================================================================================================
// Split mixer (default for the FAST shapes): the QMixer's hypernetworks read only the state (qmix.py:41-52: hyper_w_1,
// hyper_b_1, hyper_w_final, V), not the agent network, so their forward -- about two thirds of mix_td's matrix work --
// runs beside the agent recurrence, in the same launch (rec4_mixpre_kernel) on the CUs the recurrence leaves idle. Per (b, t) row it stores the
// pre-abs hyper_w_1 outputs of every agent, the pre-abs hyper_w_final outputs, hyper_b_1 and V: online on s_t, target
// on s_{t+1}; the online net also stores its layer-1 activations and the state row for the weight gradients.
// mix_td2_kernel then gathers the Qs, mixes (MixerPF::mix), forms the TD error and runs the mixer backward exactly as
// mix_td_kernel does. Same operations in the same order: bit-identical to mix_td_kernel<.., true>.
struct HypOut {
    float *on, *tg;  // [RM][hs]: w1p [N*E] | wfp [E] | b1 [E] | v (padded to 4)
    float *la, *srow;
    int hs;
};

// One 16-row tile by a pair of waves: wv 0 the target net on s_{t+1}, wv 1 the online net on s_t.
template <int HE, int E>
__device__ __forceinline__ void mix_pre_tile(const LCfg& c, const MlgBatch& bt, const MixPtrs& Mon, const MixPtrs& Mtg,
                                             const MixPack& mp, const HypOut& o, int tile, int wv, int lane) {
    using Mx = Mixer<HE, E>;
    using MP = MixerPF<HE, E, 4, MIXPF_N>;
    const int col = lane & 15, g = lane >> 4;
    const bool tgt = wv == 0;
    const int rm = tile * 16 + col;
    const int Tm = c.T - 1;
    const bool valid = rm < c.RM;
    const int b = valid ? rm / Tm : 0, t = valid ? rm % Tm : 0;
    const int N = c.N, S = c.S, NE = N * E, L1 = 2 * HE + 2 * E;
    const float* s = valid ? bt.state + (bslot(bt, b) * bt.T1 + t + (tgt ? 1 : 0)) * S : nullptr;
    floatx4 l1[Mx::L1T], w1p[MIXPF_N][Mx::TE], wfp[Mx::TE];
    float v;
    MP::hyper(tgt ? Mtg : Mon, mp, S, N, s, l1, w1p, wfp, v, lane);
    if (!valid) return;
    float* h = (tgt ? o.tg : o.on) + (int64_t)rm * o.hs;
#pragma unroll
    for (int n = 0; n < MIXPF_N; ++n) {
        if (n >= N) break;
#pragma unroll
        for (int cc = 0; cc < Mx::TE; ++cc) *reinterpret_cast<floatx4*>(h + n * E + cc * 16 + 4 * g) = w1p[n][cc];
    }
#pragma unroll
    for (int cc = 0; cc < Mx::TE; ++cc) {
        *reinterpret_cast<floatx4*>(h + NE + cc * 16 + 4 * g) = wfp[cc];
        *reinterpret_cast<floatx4*>(h + NE + E + cc * 16 + 4 * g) = l1[Mx::OB1 + cc];
    }
    if (g == 0) h[NE + 2 * E] = v;
    if (!tgt) {
        float* la = o.la + (int64_t)rm * L1;
#pragma unroll
        for (int mt = 0; mt < Mx::L1T; ++mt) *reinterpret_cast<floatx4*>(la + mt * 16 + 4 * g) = l1[mt];
        if (g == 0)
            for (int k = 0; k < S; ++k) o.srow[(int64_t)rm * S + k] = s[k];
    }
}

// The agent recurrence (agent_rec4_kernel, blocks < 2 * ntiles4) and the mixer's hypernetwork forward (mix_pre_tile,
// blockDim / 128 tiles per block after them) in one launch: the recurrence occupies (R / 4) * 2 CUs for its whole
// sequential T loop, the hypernet tiles run on the idle ones, with no cross-stream fork / join.
template <int H>
__global__ void __launch_bounds__(512) rec4_mixpre_kernel(LCfg c, AgentLayout L, const float* __restrict__ Pon,
                                                          const float* __restrict__ Ptg, const float* __restrict__ gi_on,
                                                          const float* __restrict__ gi_tg, float* __restrict__ hs_on,
                                                          float* __restrict__ hs_tg, float* __restrict__ ws_gr,
                                                          float* __restrict__ ws_gz, float* __restrict__ ws_gn,
                                                          float* __restrict__ ws_ghn, const float* __restrict__ msum,
                                                          MlgBatch bt, MixPtrs Mon, MixPtrs Mtg, MixPack mp, HypOut o) {
    const int nrec = 2 * ((c.R + 3) / 4);
    if ((int)blockIdx.x < nrec) {
        agent_rec4_body<H>(c, L, Pon, Ptg, gi_on, gi_tg, hs_on, hs_tg, ws_gr, ws_gz, ws_gn, ws_ghn, msum, blockIdx.x);
        return;
    }
    const int w = threadIdx.x >> 6, per = blockDim.x / 128;
    const int tile = ((int)blockIdx.x - nrec) * per + (w >> 1);
    if (tile * 16 >= c.RM) return;  // whole pair of waves past the last tile (block-uniform per wave pair)
    mix_pre_tile<64, 32>(c, bt, Mon, Mtg, mp, o, tile, w & 1, threadIdx.x & 63);
}

template <int HE, int E>
__global__ void __launch_bounds__(128) mix_td2_kernel(LCfg c, MlgBatch bt, MixPtrs Mon, const float* __restrict__ mac,
                                                      const float* __restrict__ tmac, const float* __restrict__ msum_p,
                                                      HypOut hy, MixOut o) {
    using Mx = Mixer<HE, E>;
    using MP = MixerPF<HE, E, 4, MIXPF_N>;
    constexpr int TE = Mx::TE, T1H = Mx::T1H;
    __shared__ float tgt_sh[16];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, col = lane & 15, g = lane >> 4;
    const int rm = blockIdx.x * 16 + col;
    const int Tm = c.T - 1;
    const bool valid = rm < c.RM;
    const int b = valid ? rm / Tm : 0, t = valid ? rm % Tm : 0;
    const int N = c.N, NE = N * E, L1 = 2 * HE + 2 * E;
    // this lane's hypernet outputs (rows past RM read row 0: finite, and their results are never stored)
    const float* h = (wv == 0 ? hy.tg : hy.on) + (int64_t)(valid ? rm : 0) * hy.hs;
    floatx4 w1c[MIXPF_N][TE], wfp[TE], b1[TE];
#pragma unroll
    for (int n = 0; n < MIXPF_N; ++n) {
        if (n >= N) break;
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) w1c[n][cc] = ld4(h + n * E + cc * 16 + 4 * g);
    }
#pragma unroll
    for (int cc = 0; cc < TE; ++cc) {
        wfp[cc] = ld4(h + NE + cc * 16 + 4 * g);
        b1[cc] = ld4(h + NE + E + cc * 16 + 4 * g);
    }
    const float vv = h[NE + 2 * E];
    // operands of the backward that depend on nothing computed here, requested now so that their L2 / HBM round
    // trips overlap the gather and the mixing (wave 1 only: wave 0 leaves after the target mix): agent 0's W_a2^T
    // block, W_f2^T, V's output row and this row's layer-1 activations (stored by mix_pre_tile)
    const float* la = hy.la + (int64_t)(valid ? rm : 0) * L1;
    floatx4 aTb[2][TE][T1H], f2w[T1H][TE], wvb[TE], lab[T1H * 2 + TE];
    auto load_aT = [&](int n, floatx4 (&d)[TE][T1H]) {
#pragma unroll
        for (int cc = 0; cc < TE; ++cc)
#pragma unroll
            for (int mt = 0; mt < T1H; ++mt) d[cc][mt] = ld4(Mon.a2T + (int64_t)(mt * 16 + col) * NE + n * E + cc * 16 + 4 * g);
    };
    if (wv == 1) {
        load_aT(0, aTb[0]);
#pragma unroll
        for (int mt = 0; mt < T1H; ++mt)
#pragma unroll
            for (int cc = 0; cc < TE; ++cc) f2w[mt][cc] = ld4(Mon.f2T + (int64_t)(mt * 16 + col) * E + cc * 16 + 4 * g);
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) wvb[cc] = ld4(Mon.v2p + cc * 16 + 4 * g);
#pragma unroll
        for (int mt = 0; mt < T1H; ++mt) {
            lab[mt] = ld4(la + (Mx::OW1 + mt) * 16 + 4 * g);
            lab[T1H + mt] = ld4(la + (Mx::OWF + mt) * 16 + 4 * g);
        }
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) lab[2 * T1H + cc] = ld4(la + (Mx::OVH + cc) * 16 + 4 * g);
    }
    float cq[MAXN], tq[MAXN];
    for (int n = 0; n < N; ++n) cq[n] = tq[n] = 0.f;
    gather_q_rows<MIXPF_A>(c, bt, mac, tmac, b, t, valid, g, cq, tq);
    floatx4 pre[TE], hid[TE];
    if (wv == 0) {
        const float tv = MP::mix(N, tq, b1, w1c, wfp, vv, pre, hid);
        if (g == 0) tgt_sh[col] = tv;
    }
    const float m = (valid && t < t_eff(msum_p) - 1) ? mask_at(bt, b, t) : 0.f;  // reference truncation
    const float rwd = valid ? bt.reward[bslot(bt, b) * bt.T1 + t] : 0.f;
    const float term = valid ? (float)bt.terminated[bslot(bt, b) * bt.T1 + t] : 0.f;
    const float msum = msum_p[0];
    float qtot = 0.f;
    if (wv == 1) qtot = MP::mix(N, cq, b1, w1c, wfp, vv, pre, hid);
    __syncthreads();
    if (wv == 0) return;
    const float tgt = tgt_sh[col];
    const float y = rwd + c.gamma * (1.f - term) * tgt;  // q_learner.py:86
    const float mtd = (qtot - y) * m;                     // :89-95
    const float dy = 2.f * mtd * m / msum;                // d loss / d q_tot
    {
        float p0 = g == 0 ? mtd * mtd : 0.f, p1 = g == 0 ? fabsf(mtd) : 0.f;
        float p2 = g == 0 ? qtot * m : 0.f, p3 = g == 0 ? y * m : 0.f;
        p0 = row_sum16(p0);
        p1 = row_sum16(p1);
        p2 = row_sum16(p2);
        p3 = row_sum16(p3);
        if (lane == 0) {
            float* pp = o.part + (int64_t)blockIdx.x * 4;
            pp[0] = p0;
            pp[1] = p1;
            pp[2] = p2;
            pp[3] = p3;
        }
    }
    // ---- QMixer backward (autograd of qmix.py:41-59), as mix_td_kernel ----
    floatx4 dpre[TE], dwf[TE];
#pragma unroll
    for (int cc = 0; cc < TE; ++cc) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float dh = dy * fabsf(wfp[cc][q]);
            const float sg = wfp[cc][q] > 0.f ? 1.f : (wfp[cc][q] < 0.f ? -1.f : 0.f);
            dwf[cc][q] = dy * hid[cc][q] * sg;
            dpre[cc][q] = pre[cc][q] > 0.f ? dh : dh * (hid[cc][q] + 1.f);
        }
    }
    floatx4 dw1h[T1H];
#pragma unroll
    for (int mt = 0; mt < T1H; ++mt) dw1h[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
    float dq[MAXN];
#pragma unroll
    for (int n = 0; n < MIXPF_N; ++n) {  // N <= MIXPF_N (the FAST shapes): static ping-pong buffers
        if (n >= N) break;
        if (n + 1 < MIXPF_N && n + 1 < N) load_aT(n + 1, aTb[(n + 1) & 1]);
        const floatx4(&aT)[TE][T1H] = aTb[n & 1];
        float part = 0.f;
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) {
            const floatx4 wp = w1c[n][cc];
            floatx4 dlt;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                part += fabsf(wp[q]) * dpre[cc][q];
                const float sg = wp[q] > 0.f ? 1.f : (wp[q] < 0.f ? -1.f : 0.f);
                dlt[q] = cq[n] * dpre[cc][q] * sg;
            }
            if (valid) *reinterpret_cast<floatx4*>(o.da2 + (int64_t)rm * NE + n * E + cc * 16 + 4 * g) = dlt;
#pragma unroll
            for (int mt = 0; mt < T1H; ++mt) dw1h[mt] = mfma_chunk(aT[cc][mt], dlt, dw1h[mt]);
        }
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
        dq[n] = part;
    }
    floatx4 dwfh[T1H];
#pragma unroll
    for (int mt = 0; mt < T1H; ++mt) {
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) acc = mfma_chunk(f2w[mt][cc], dwf[cc], acc);
        dwfh[mt] = acc;
    }
    if (valid) {
        // layer-1 activations (stored by mix_pre_tile, loaded above) for the ReLU masks
        float* d1 = o.d1 + (int64_t)rm * L1;
#pragma unroll
        for (int mt = 0; mt < T1H; ++mt) {  // w1h
            const floatx4 l = lab[mt];
            floatx4 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = l[q] > 0.f ? dw1h[mt][q] : 0.f;
            *reinterpret_cast<floatx4*>(d1 + mt * 16 + 4 * g) = v;
        }
#pragma unroll
        for (int mt = 0; mt < T1H; ++mt) {  // wfh
            const floatx4 l = lab[T1H + mt];
            floatx4 acc = dwfh[mt];
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] = l[q] > 0.f ? acc[q] : 0.f;
            *reinterpret_cast<floatx4*>(d1 + HE + mt * 16 + 4 * g) = acc;
        }
#pragma unroll
        for (int cc = 0; cc < TE; ++cc) {  // b1, vh
            *reinterpret_cast<floatx4*>(d1 + 2 * HE + cc * 16 + 4 * g) = dpre[cc];
            const floatx4 wv = wvb[cc];
            const floatx4 l = lab[2 * T1H + cc];
            floatx4 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = l[q] > 0.f ? dy * wv[q] : 0.f;
            *reinterpret_cast<floatx4*>(d1 + 2 * HE + E + cc * 16 + 4 * g) = v;
            *reinterpret_cast<floatx4*>(o.df2 + (int64_t)rm * E + cc * 16 + 4 * g) = dwf[cc];
        }
        if (g == 0) o.dv2[rm] = dy;
    }
    if (valid && g == 0) {  // dQ per agent row (t-major) and its one-hot expansion for dW2 (d2 zeroed by prep_kernel:
                            // whole-row writes here measured 3.7 us slower, and the zeroing is off prep's critical path)
        for (int n = 0; n < N; ++n) {
            const int r = b * N + n;
            o.dq[(int64_t)t * c.R + r] = dq[n];
            const int a = (int)bt.actions[(bslot(bt, b) * bt.T1 + t) * N + n];
            o.d2[((int64_t)t * c.R + r) * c.A + a] = dq[n];
        }
    }
}

// ================================================================================================
// reverse-time GRU backward; wave w owns hidden chunk w. W_hh^T rows of the chunk live in VGPRs, the
// step's gate values are prefetched one step ahead, dGH is exchanged through LDS (double buffered).
// dh_{t-1} = dh * z + W_hh^T dGH.  dX = W_ih^T dGI does not feed the recurrence: agent_dx_kernel.
template <int H>
__global__ void __launch_bounds__(512) agent_bwd_kernel(LCfg c, MlgBatch bt, AgentLayout L, const float* __restrict__ P,
                                                        const float* __restrict__ ws_hs, const float* __restrict__ ws_gr,
                                                        const float* __restrict__ ws_gz, const float* __restrict__ ws_gn,
                                                        const float* __restrict__ ws_ghn, const float* __restrict__ dqv,
                                                        float* __restrict__ dgi, float* __restrict__ dgh,
                                                        const float* __restrict__ msum) {
    constexpr int LDG = 3 * H + 4;
    constexpr int KC = 3 * H / 16;
    __shared__ __attribute__((aligned(16))) float sgh[2][16 * LDG];
    __shared__ __attribute__((aligned(16))) float w2s[MLG_BWD_MAXA * H];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int col = lane & 15, g = lane >> 4;
    const int r = blockIdx.x * 16 + col;
    const bool valid = r < c.R;
    const int b = valid ? r / c.N : 0, n = valid ? r % c.N : 0;
    const int R = c.R, N = c.N;
    const int f0 = w * 16 + 4 * g;
    // A operand of W_hh^T: row = feature w*16 + col, K = gate-row k: W_hh[k][feature]
    floatx4 wt[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int q = 0; q < 4; ++q) wt[kc][q] = P[L.whh + (int64_t)(kc * 16 + 4 * g + q) * H + w * 16 + col];
    const int rr = valid ? r : 0;
    for (int i = tid; i < c.A * H; i += blockDim.x) w2s[i] = P[L.w2 + i];  // fc2 rows for dh += dq W2[a]
    const int64_t abase = bslot(bt, b) * bt.T1 * N + n;  // loop-invariant: no dependent slot-map load per step
    struct Step {
        floatx4 rg, zg, ng, ghn, hp;
        float dq;
        int a;
    };
    auto load_step = [&](int t, Step& s) {
        const int64_t o = ((int64_t)t * R + rr) * H + f0;
        s.rg = ld4(ws_gr + o);
        s.zg = ld4(ws_gz + o);
        s.ng = ld4(ws_gn + o);
        s.ghn = ld4(ws_ghn + o);
        s.hp = ld4(ws_hs + o);  // HS[t] = h_{t-1}
        const int tq = t < c.T - 1 ? t : c.T - 2;  // unconditional (clamped) loads; dq / action unused at T-1
        s.dq = dqv[(int64_t)tq * R + rr];
        s.a = t < c.T - 1 ? (int)bt.actions[abase + (int64_t)tq * N] : -1;
    };
    const int Te = t_eff(msum);
    if (valid) {  // steps past max_t_filled: zero deltas (wgrad rows)
        for (int t = Te; t < c.T; ++t) {
            const int64_t o3 = ((int64_t)t * R + r) * 3 * H + f0;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                *reinterpret_cast<floatx4*>(dgi + o3 + q * H) = floatx4{0.f, 0.f, 0.f, 0.f};
                *reinterpret_cast<floatx4*>(dgh + o3 + q * H) = floatx4{0.f, 0.f, 0.f, 0.f};
            }
        }
    }
    floatx4 dh = {0.f, 0.f, 0.f, 0.f};
    // a step's saved gates are prefetched one step ahead into ping-pong registers (2x-unrolled loop, no copies:
    // the wait for them never covers the previous step's stores); W2 rows come from LDS, not a dependent load
    const __amdgpu_buffer_rsrc_t rs_gi = mlg_rsrc(dgi), rs_gh = mlg_rsrc(dgh);
    auto step = [&](int t, const Step& s, Step& nx, int cur) {
        load_step(t > 0 ? t - 1 : 0, nx);
        if (valid && s.a >= 0) dh += s.dq * ld4(w2s + s.a * H + f0);
        floatx4 drp, dzp, dnp, dghn, dhd;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float dn = dh[q] * (1.f - s.zg[q]);
            const float dz = dh[q] * (s.hp[q] - s.ng[q]);
            dhd[q] = dh[q] * s.zg[q];
            dnp[q] = dn * (1.f - s.ng[q] * s.ng[q]);
            const float dr = dnp[q] * s.ghn[q];
            drp[q] = dr * s.rg[q] * (1.f - s.rg[q]);
            dzp[q] = dz * s.zg[q] * (1.f - s.zg[q]);
            dghn[q] = dnp[q] * s.rg[q];
        }
        float* gh = sgh[cur] + col * LDG;
        *reinterpret_cast<floatx4*>(gh + f0) = drp;
        *reinterpret_cast<floatx4*>(gh + H + f0) = dzp;
        *reinterpret_cast<floatx4*>(gh + 2 * H + f0) = dghn;
        const int64_t o3 = ((int64_t)t * R + r) * 3 * H + f0;
        st4_if(rs_gi, o3, drp, valid);
        st4_if(rs_gi, o3 + H, dzp, valid);
        st4_if(rs_gi, o3 + 2 * H, dnp, valid);
        st4_if(rs_gh, o3, drp, valid);
        st4_if(rs_gh, o3 + H, dzp, valid);
        st4_if(rs_gh, o3 + 2 * H, dghn, valid);
        __syncthreads();
        floatx4 dprev = dhd;
        const float* ghr = sgh[cur] + col * LDG + 4 * g;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) dprev = mfma_chunk(wt[kc], ld4(ghr + kc * 16), dprev);
        dh = dprev;
    };
    Step sa, sb;
    load_step(Te - 1, sa);
    step(Te - 1, sa, sb, 0);  // peeled (see agent_rec_kernel)
    for (int t = Te - 2; t >= 0; t -= 2) {
        step(t, sb, sa, 1);
        if (t > 0) step(t - 1, sa, sb, 0);
    }
}

// The backward recurrence on 4-row tiles (v_mfma_f32_4x4x1_16b_f32, as agent_rec4_kernel). Wave w owns hidden
// features 16w..16w+15; block b = 4kq + fg accumulates W_hh^T dGH for features 16w + 4fg + i over the K quarter
// kq (48 of the 3H gate rows, W_hh columns in VGPRs). The four quarter partials are summed across the wave's
// 16-lane rows with a transposing reduction (rows_sum_transpose4): lane (row kq, fg, j) ends up owning feature
// 16w + 4fg + kq of row j, so all 64 lanes run the elementwise GRU backward, one (feature, row) each.
// grid (ntiles4), H/16 waves.
template <int H>
__global__ void __launch_bounds__(512) agent_bwd4_kernel(LCfg c, MlgBatch bt, AgentLayout L, const float* __restrict__ P,
                                                         const float* __restrict__ ws_hs, const float* __restrict__ ws_gr,
                                                         const float* __restrict__ ws_gz, const float* __restrict__ ws_gn,
                                                         const float* __restrict__ ws_ghn, const float* __restrict__ dqv,
                                                         float* __restrict__ dgi, float* __restrict__ dgh,
                                                         const float* __restrict__ msum) {
    LStamps lst;
    lst.init();
    const int r = blockIdx.x * 4 + ((threadIdx.x & 63) & 3);
    const bool valid = r < c.R;
    const int b = valid ? r / c.N : 0, n = valid ? r % c.N : 0;
    const mlg::Gru4Bwd a{c.R, c.T, c.A, c.N, P + L.whh, P + L.w2, ws_hs, ws_gr, ws_gz, ws_gn, ws_ghn, dqv,
                         bt.actions, dgi, dgh};
    mlg::gru4_bwd<H>(a, blockIdx.x, t_eff(msum), bslot(bt, b) * bt.T1 * c.N + n, lst);
    lst.flush(1);
}

// The reverse recurrence (blocks < nbwd, H = 64: 4 waves each) and, as the launch's remaining workgroups, the weight
// gradients whose deltas are final after the mixer kernel (fc2 and the mixer's jobs: table view JA). The
// recurrence keeps 40 CUs busy for its 101 sequential steps; the wgrad workgroups fill the others, with no second
// stream and no events (each event record costs a few us of queue time). Same per-job arithmetic as the separate
// launches.
template <int H>
__global__ void __launch_bounds__(256, 2) bwd4_wgrad_kernel(LCfg c, MlgBatch bt, AgentLayout L, const float* __restrict__ P,
                                                         const float* __restrict__ ws_hs, const float* __restrict__ ws_gr,
                                                         const float* __restrict__ ws_gz, const float* __restrict__ ws_gn,
                                                         const float* __restrict__ ws_ghn, const float* __restrict__ dqv,
                                                         float* __restrict__ dgi, float* __restrict__ dgh,
                                                         const float* __restrict__ msum, WJobs JA,
                                                         float* __restrict__ slab, int nbwd) {
    if ((int)blockIdx.x >= nbwd) {
        mlg::wgrad_block_body<16>(JA, slab, (int)blockIdx.x - nbwd);
        return;
    }
    LStamps lst;
    lst.init();
    const int r = blockIdx.x * 4 + ((threadIdx.x & 63) & 3);
    const bool valid = r < c.R;
    const int b = valid ? r / c.N : 0, n = valid ? r % c.N : 0;
    const mlg::Gru4Bwd a{c.R, c.T, c.A, c.N, P + L.whh, P + L.w2, ws_hs, ws_gr, ws_gz, ws_gn, ws_ghn, dqv,
                         bt.actions, dgi, dgh};
    mlg::gru4_bwd<H>(a, blockIdx.x, t_eff(msum), bslot(bt, b) * bt.T1 * c.N + n, lst);
    lst.flush(1);
}

// dA = (W_ih^T dGI) * (x > 0) for every (t, row): grid (ntiles, T), HC waves (wave = feature chunk).
template <int H>
__global__ void __launch_bounds__(512) agent_dx_kernel(LCfg c, const float* __restrict__ wihT,
                                                       const float* __restrict__ ws_x, const float* __restrict__ dgi,
                                                       float* __restrict__ da, const float* __restrict__ msum) {
    const int tile = blockIdx.x, t = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int col = lane & 15, g = lane >> 4;
    const int r = tile * 16 + col;
    const bool valid = r < c.R;
    if (t >= t_eff(msum)) {
        if (valid)
            *reinterpret_cast<floatx4*>(da + ((int64_t)t * c.R + r) * H + w * 16 + 4 * g) = floatx4{0.f, 0.f, 0.f, 0.f};
        return;
    }
    const int64_t row = (int64_t)t * c.R + (valid ? r : 0);
    const float* wrow = wihT + (int64_t)(w * 16 + col) * 3 * H + 4 * g;
    const float* grow = dgi + row * 3 * H + 4 * g;
    const int64_t o = row * H + w * 16 + 4 * g;
    const floatx4 xv = ld4(ws_x + o);  // the ReLU mask, requested with the operands (row 0 for padding lanes)
    floatx4 dx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < 3 * H / 16; ++kc) dx = mfma_chunk(ld4(wrow + kc * 16), ld4(grow + kc * 16), dx);
    if (valid) {
#pragma unroll
        for (int q = 0; q < 4; ++q) dx[q] = xv[q] > 0.f ? dx[q] : 0.f;
        *reinterpret_cast<floatx4*>(da + o) = dx;
    }
}

// ================================================================================================
// clip_grad_norm_ + RMSprop over all parameters (grid-wide; every block derives the same norm from the
// per-block partials in a fixed order), loss/stat reduction in block 0.
__global__ void __launch_bounds__(1024) finish_kernel(const float* __restrict__ part, int n_part,
                                                      const float* __restrict__ msum_p, float* __restrict__ params,
                                                      float* __restrict__ grads, float* __restrict__ sq, int64_t n_params,
                                                      float lr, float alpha, float eps, float max_norm, int N,
                                                      float* __restrict__ stats, const float* __restrict__ nrm_part,
                                                      int n_nrm, float* __restrict__ tsync, double* __restrict__ trained) {
    __shared__ float red[1024];
    const int tid = threadIdx.x;
    // this thread's parameter, gradient and square average, requested before the norm reduction they wait for
    const int64_t ip = (int64_t)blockIdx.x * blockDim.x + tid;
    const bool has = ip < n_params;
    const float g0 = has ? grads[ip] : 0.f, sq0 = has ? sq[ip] : 0.f, p0 = has ? params[ip] : 0.f;
    float s = 0.f;
    for (int i = tid; i < n_nrm; i += blockDim.x) s += nrm_part[i];
    const float norm = sqrtf(block_sum_1024(s, red));
    const float coef = fminf(max_norm / (norm + 1e-6f), 1.f);  // torch clip_grad_norm_ (clamped coef)
    if (has) {
        const float gi = g0 * coef;
        grads[ip] = gi;
        const float a = alpha * sq0 + (1.f - alpha) * gi * gi;  // RMSprop square_avg
        sq[ip] = a;
        const float pn = p0 - lr * gi / (sqrtf(a) + eps);
        params[ip] = pn;
        if (tsync) tsync[ip] = pn;  // target update due after this step (q_learner.py:127-128), same launch
    }
    // the four stat sums on blocks 0..3 (one each, same order as one block doing all four: bit-identical), so no
    // block runs four block reductions after its parameter slice
    const float ms = msum_p[0];
    for (int k = blockIdx.x; k < 4; k += gridDim.x) {
        float v = 0.f;
        for (int j = tid; j < n_part; j += blockDim.x) v += part[(int64_t)j * 4 + k];
        const float sk = block_sum_1024(v, red);
        if (tid == 0) {
            if (k == 0) stats[0] = sk / ms;
            else if (k == 1) stats[2] = sk / ms;
            else stats[k + 1] = sk / (ms * N);  // k = 2, 3: stats[3], stats[4] (per agent)
        }
    }
    if (blockIdx.x == 0 && tid == 0) {
        stats[1] = norm;
        stats[5] = ms;
        stats[6] = ms;
        stats[7] = 0.f;
        if (trained) trained[0] += (double)ms;  // Agent.trained_steps (q_learner.py:104)
    }
}

// ================================================================================================
// host side
struct Plan {
    LCfg c;
    AgentLayout L;
    AgentOffs ao;
    MixOffs mo;
    MixPack mp;
    WsLayout w;
    int64_t n_agent, n_mixer;
};

int check_cfg(const MlgLearnerCfg* c) {
    MLG_REQUIRE(c != nullptr, "null learner cfg");
    MLG_REQUIRE(c->H == 32 || c->H == 64 || c->H == 128, "rnn_hidden_dim=%d unsupported (32/64/128)", c->H);
    MLG_REQUIRE(c->B >= 1 && c->T >= 2 && c->N >= 1 && c->N <= MAXN && c->A >= 1, "learner: bad sizes B=%d T=%d N=%d",
                c->B, c->T, c->N);
    MLG_REQUIRE(c->A <= MLG_BWD_MAXA, "learner: n_actions=%d > %d unsupported", c->A, MLG_BWD_MAXA);
    MLG_REQUIRE((int64_t)c->T * c->B * c->N * 3 * c->H < (int64_t)1 << 29,
                "learner: T*B*N*3H=%lld floats exceeds the 2 GB buffer-store range",
                (long long)c->T * c->B * c->N * 3 * c->H);
    MLG_REQUIRE(c->mixer == 1 || c->mixer == 2, "learner: mixer must be vdn or qmix (IQL is not built)");
    if (c->mixer == 2) {
        MLG_REQUIRE(c->hypernet_layers == 2, "learner: qmix hypernet_layers=%d unsupported (2)", c->hypernet_layers);
        MLG_REQUIRE(c->E == 32 && c->HE == 64, "learner: qmix mixing_embed_dim=32, hypernet_embed=64 supported (got %d, %d)",
                    c->E, c->HE);
    }
    return 0;
}

Plan make_plan(const MlgLearnerCfg* cfg, int T1) {
    Plan p;
    LCfg& c = p.c;
    c.B = cfg->B;
    c.T = cfg->T;
    c.T1 = T1;
    c.N = cfg->N;
    c.A = cfg->A;
    c.Ap = (cfg->A + 15) / 16 * 16;
    c.d_obs = cfg->d_obs;
    c.d_in = cfg->d_obs + (cfg->obs_last_action ? cfg->A : 0) + (cfg->obs_agent_id ? cfg->N : 0);
    c.H = cfg->H;
    c.S = cfg->S;
    c.E = cfg->E;
    c.HE = cfg->HE;
    c.mixer = cfg->mixer;
    c.double_q = cfg->double_q;
    c.last_action = cfg->obs_last_action;
    c.agent_id = cfg->obs_agent_id;
    c.R = cfg->B * cfg->N;
    c.RM = cfg->B * (cfg->T - 1);
    c.gamma = cfg->gamma;
    MlgAgentDims d{cfg->d_obs, cfg->A, cfg->N, cfg->H, c.d_in, cfg->obs_last_action, cfg->obs_agent_id};
    p.L = make_agent_layout(d);
    p.ao = agent_offs(c.H, c.d_in, c.A);
    p.mo = mix_offs(c.N, c.S, c.E, c.HE);
    p.mp = mix_pack(c.N, c.S, c.E, c.HE);
    p.n_agent = p.ao.total;
    p.n_mixer = c.mixer == 2 ? p.mo.total : 0;
    WsLayout& w = p.w;
    const int64_t T = c.T, R = c.R, H = c.H, RM = c.RM;
    const int L1 = 2 * c.HE + 2 * c.E;
    int64_t o = 0;
    auto take = [&](int64_t n) { int64_t r = o; o += a4(n); return r; };
    w.p_on = take(p.L.total);
    w.p_tg = take(p.L.total);
    w.wihT = take(3 * H * H);
    w.mix_on = take(p.mp.total);
    w.mix_tg = take(p.mp.total);
    w.in = take(T * R * c.d_in);
    w.x = take(T * R * H);
    w.hs = take((T + 1) * R * H);
    w.hs_tg = take((T + 1) * R * H);
    w.gi_on = take(T * R * 3 * H);
    w.gi_tg = take(T * R * 3 * H);
    w.gr = take(T * R * H);
    w.gz = take(T * R * H);
    w.gn = take(T * R * H);
    w.ghn = take(T * R * H);
    w.mac = take(T * R * c.A);
    w.tmac = take(T * R * c.A);
    w.dq = take(T * R);
    w.d2 = take(T * R * c.A);
    w.dgi = take(T * R * 3 * H);
    w.dgh = take(T * R * 3 * H);
    w.da = take(T * R * H);
    w.srow = take(RM * c.S);
    w.l1act = take(RM * L1);
    w.d1 = take(RM * L1);
    w.da2 = take(RM * c.N * c.E);
    w.df2 = take(RM * c.E);
    w.dv2 = take(RM);
    w.hyp_stride = c.mixer == 2 ? (int)a4((int64_t)c.N * c.E + 2 * c.E + 1) : 0;  // mix_pre_tile rows (HypOut)
    w.hyp_on = take(RM * w.hyp_stride);
    w.hyp_tg = take(RM * w.hyp_stride);
    w.n_mix_tiles = (int)((RM + 15) / 16);
    w.part = take((int64_t)w.n_mix_tiles * 4);
    w.msum = take(4);
    w.rows = take(MLG_INLINE_ROWS);
    w.nrm = 0;  // placed after the slab (size known once the jobs are built)
    w.slab = o;
    w.total = o;  // + slab size, filled by make_jobs
    return p;
}


// builds the job list; with ws == nullptr only sizes are computed (pointers are offsets from 0)
WJobs make_jobs(Plan& p, float* ws, float* grads, int64_t* slab_floats, int* n_tasks, int64_t* n_red) {
    const LCfg& c = p.c;
    float* W = ws ? ws : nullptr;
    auto at = [&](int64_t off) { return W ? W + off : (float*)nullptr; };
    float* G = grads;
    auto gp = [&](int64_t off) { return G ? G + off : (float*)nullptr; };
    const int TR = c.T * c.R, H = c.H, L1 = 2 * c.HE + 2 * c.E, RM = c.RM;
    WJobs J;
    J.n = 0;
    const AgentOffs& a = p.ao;
    J.j[J.n++] = mlg::bjob(at(p.w.da), H, at(p.w.in), c.d_in, gp(a.fc1w), gp(a.fc1b), H, c.d_in, TR);
    J.j[J.n++] = mlg::bjob(at(p.w.dgi), 3 * H, at(p.w.x), H, gp(a.wih), gp(a.bih), 3 * H, H, TR);
    J.j[J.n++] = mlg::bjob(at(p.w.dgh), 3 * H, at(p.w.hs), H, gp(a.whh), gp(a.bhh), 3 * H, H, TR);
    J.j[J.n++] = mlg::bjob(at(p.w.d2), c.A, at(p.w.hs) ? at(p.w.hs) + (int64_t)c.R * H : nullptr, H, gp(a.fc2w), gp(a.fc2b),
                     c.A, H, TR);
    if (c.mixer == 2) {
        const MixOffs& m = p.mo;
        const int64_t G0 = p.n_agent;
        auto mg = [&](int64_t off) { return G ? G + G0 + off : (float*)nullptr; };
        const float* d1 = at(p.w.d1);
        const float* la = at(p.w.l1act);
        auto off = [&](const float* base, int64_t k) { return base ? base + k : (const float*)nullptr; };
        J.j[J.n++] = mlg::bjob(off(d1, 0), L1, at(p.w.srow), c.S, mg(m.w1_0w), mg(m.w1_0b), c.HE, c.S, RM);
        J.j[J.n++] = mlg::bjob(off(d1, c.HE), L1, at(p.w.srow), c.S, mg(m.wf_0w), mg(m.wf_0b), c.HE, c.S, RM);
        J.j[J.n++] = mlg::bjob(off(d1, 2 * c.HE), L1, at(p.w.srow), c.S, mg(m.b1w), mg(m.b1b), c.E, c.S, RM);
        J.j[J.n++] = mlg::bjob(off(d1, 2 * c.HE + c.E), L1, at(p.w.srow), c.S, mg(m.v0w), mg(m.v0b), c.E, c.S, RM);
        J.j[J.n++] = mlg::bjob(at(p.w.da2), (int64_t)c.N * c.E, off(la, 0), L1, mg(m.w1_2w), mg(m.w1_2b), c.N * c.E, c.HE, RM);
        J.j[J.n++] = mlg::bjob(at(p.w.df2), c.E, off(la, c.HE), L1, mg(m.wf_2w), mg(m.wf_2b), c.E, c.HE, RM);
        J.j[J.n++] = mlg::bjob(at(p.w.dv2), 1, off(la, 2 * c.HE + c.E), L1, mg(m.v2w), mg(m.v2b), 1, c.E, RM);
    }
    int64_t slab_part;
    *slab_floats = mlg::layout_bjobs(J, n_tasks, n_red, &slab_part);  // slab partials + per-block norm partials
    p.w.nrm = p.w.slab + slab_part;
    return J;
}

template <int H>
int run_train(Plan& p, const MlgLearnerCfg* cfg, const MlgLearnerBufs* bufs, hipStream_t s) {
    const LCfg& c = p.c;
    float* ws = bufs->workspace;
    MlgBatch bt = bufs->batch;
    int32_t* rows_ws = reinterpret_cast<int32_t*>(ws + p.w.rows);
    if (bufs->host_rows) bt.rows = rows_ws;  // filled by prep_kernel's block 0 from its argument
    const float* params = bufs->params;
    const float* tparams = bufs->target_params;
    // ---- fused prologue: pack online / target agent + mixer, W_ih^T, zero d2 / dq, mask sum ----
    auto agent_ptrs = [&](const float* flat) {
        return MlgAgentParams{flat + p.ao.fc1w, flat + p.ao.fc1b, flat + p.ao.wih, flat + p.ao.bih,
                              flat + p.ao.whh, flat + p.ao.bhh, flat + p.ao.fc2w, flat + p.ao.fc2b};
    };
    PrepJob pj;
    pj.L = p.L;
    pj.ap_on = agent_ptrs(params);
    pj.ap_tg = agent_ptrs(tparams);
    pj.p_on = ws + p.w.p_on;
    pj.p_tg = ws + p.w.p_tg;
    pj.wih = params + p.ao.wih;
    pj.wihT = ws + p.w.wihT;
    pj.rows3 = 3 * c.H;
    pj.cols = c.H;
    pj.mp = p.mp;
    pj.mo = p.mo;
    pj.mix_src_on = params + p.n_agent;
    pj.mix_src_tg = tparams + p.n_agent;
    pj.mix_on = ws + p.w.mix_on;
    pj.mix_tg = ws + p.w.mix_tg;
    pj.N = c.N;
    pj.S = c.S;
    pj.E = c.E;
    pj.HE = c.HE;
    pj.mixer = c.mixer;
    // split mixer (default for the FAST shapes): the hypernetwork forward rides in the recurrence launch
    // (rec4_mixpre_kernel), mix_td2_kernel does the rest; MLG_MIX_FUSED=1: the one-kernel mix_td
    static const bool rec16 = getenv("MLG_LEARNER_REC16") != nullptr;  // A/B switch: the 16-row tile recurrence
    const bool fast_mix = p.mp.Sp <= 64 && c.N <= MIXPF_N && c.A <= MIXPF_A && !getenv("MLG_MIX_GENERIC");
    static const bool fused_env = getenv("MLG_MIX_FUSED") != nullptr;
    const int threads = (c.H / 16) * 64;
    const bool split_mix = c.mixer == 2 && fast_mix && !fused_env && !rec16 && threads % 128 == 0;
    pj.d2 = ws + p.w.d2;  // d2 is sparse: zero it (and dq) every call
    pj.dq = ws + p.w.dq;
    pj.n_d2 = (int64_t)c.T * c.R * c.A;
    pj.n_dq = (int64_t)c.T * c.R;
    pj.bt = bt;
    pj.B = c.B;
    pj.T = c.T;
    pj.msum = ws + p.w.msum;
    pj.n_rows_in = 0;
    pj.rows_dst = rows_ws;
    if (bufs->host_rows) {
        pj.n_rows_in = c.B;
        for (int b = 0; b < c.B; ++b) pj.rows_in[b] = bufs->host_rows[b];
    }
    {
        const int64_t work = 2 * p.L.total + 3 * (int64_t)c.H * c.H + (c.mixer == 2 ? 2 * p.mp.total : 0) + pj.n_d2 + pj.n_dq;
        const int blocks = 1 + (int)std::min<int64_t>((work + 1023) / 1024, 512);
        hipLaunchKernelGGL(prep_kernel, dim3(blocks), dim3(1024), 0, s, pj);
    }
    MixPtrs Mon{}, Mtg{};
    if (c.mixer == 2) {
        const int64_t g0 = p.n_agent;
        auto ptrs = [&](const float* flat, const float* pk) {
            MixPtrs m;
            m.m1 = pk + p.mp.m1;
            m.mb1 = pk + p.mp.mb1;
            m.a2 = flat + g0 + p.mo.w1_2w;
            m.ba2 = flat + g0 + p.mo.w1_2b;
            m.a2T = pk + p.mp.a2T;
            m.f2 = flat + g0 + p.mo.wf_2w;
            m.bf2 = flat + g0 + p.mo.wf_2b;
            m.f2T = pk + p.mp.f2T;
            m.v2p = pk + p.mp.v2p;
            m.bv2p = pk + p.mp.bv2p;
            return m;
        };
        Mon = ptrs(params, ws + p.w.mix_on);
        Mtg = ptrs(tparams, ws + p.w.mix_tg);
    }
    const int ntiles = (c.R + 15) / 16;
    HypOut hy{ws + p.w.hyp_on, ws + p.w.hyp_tg, ws + p.w.l1act, ws + p.w.srow, p.w.hyp_stride};
    hipLaunchKernelGGL((agent_in_kernel<H>), dim3(ntiles, c.T, 2), dim3(threads), 0, s, c, bt, p.L, ws + p.w.p_on,
                       ws + p.w.p_tg, ws + p.w.in, ws + p.w.x, ws + p.w.gi_on, ws + p.w.gi_tg, ws + p.w.msum);
    if (split_mix) {
        const int nrec = 2 * ((c.R + 3) / 4), per = threads / 128;
        hipLaunchKernelGGL((rec4_mixpre_kernel<H>), dim3(nrec + (p.w.n_mix_tiles + per - 1) / per), dim3(threads), 0, s,
                           c, p.L, ws + p.w.p_on, ws + p.w.p_tg, ws + p.w.gi_on, ws + p.w.gi_tg, ws + p.w.hs,
                           ws + p.w.hs_tg, ws + p.w.gr, ws + p.w.gz, ws + p.w.gn, ws + p.w.ghn, ws + p.w.msum, bt, Mon,
                           Mtg, p.mp, hy);
    } else if (rec16)
        hipLaunchKernelGGL((agent_rec_kernel<H>), dim3(2 * ntiles), dim3(threads), 0, s, c, p.L, ws + p.w.p_on,
                           ws + p.w.p_tg, ws + p.w.gi_on, ws + p.w.gi_tg, ws + p.w.hs, ws + p.w.hs_tg, ws + p.w.gr,
                           ws + p.w.gz, ws + p.w.gn, ws + p.w.ghn, ws + p.w.msum);
    else
        hipLaunchKernelGGL((agent_rec4_kernel<H>), dim3(2 * ((c.R + 3) / 4)), dim3(threads), 0, s, c, p.L,
                           ws + p.w.p_on, ws + p.w.p_tg, ws + p.w.gi_on, ws + p.w.gi_tg, ws + p.w.hs, ws + p.w.hs_tg,
                           ws + p.w.gr, ws + p.w.gz, ws + p.w.gn, ws + p.w.ghn, ws + p.w.msum);
    hipLaunchKernelGGL((agent_q_kernel<H>), dim3(ntiles, c.T, 2), dim3(64 * (c.Ap / 16)), 0, s, c, p.L, ws + p.w.p_on,
                       ws + p.w.p_tg, ws + p.w.hs, ws + p.w.hs_tg, ws + p.w.mac, ws + p.w.tmac, ws + p.w.msum);
    MixOut mo{ws + p.w.srow, ws + p.w.l1act, ws + p.w.d1, ws + p.w.da2, ws + p.w.df2, ws + p.w.dv2,
              ws + p.w.dq, ws + p.w.d2, ws + p.w.part};
    if (split_mix) {
        hipLaunchKernelGGL((mix_td2_kernel<64, 32>), dim3(p.w.n_mix_tiles), dim3(128), 0, s, c, bt, Mon, ws + p.w.mac,
                           ws + p.w.tmac, ws + p.w.msum, hy, mo);
    } else if (fast_mix)
        hipLaunchKernelGGL((mix_td_kernel<64, 32, true>), dim3(p.w.n_mix_tiles), dim3(128), 0, s, c, bt, Mon, Mtg, p.mp,
                           ws + p.w.mac, ws + p.w.tmac, ws + p.w.msum, mo);
    else
        hipLaunchKernelGGL((mix_td_kernel<64, 32>), dim3(p.w.n_mix_tiles), dim3(128), 0, s, c, bt, Mon, Mtg, p.mp,
                           ws + p.w.mac, ws + p.w.tmac, ws + p.w.msum, mo);
    // weight gradients: fc2 and the mixer's jobs (final after the mixer kernel, table view JA) run as extra
    // workgroups of the reverse-recurrence launch (H = 64, bwd4_wgrad_kernel); fc1 / W_ih / W_hh (view JB) after
    // agent_dx; one reduce over the whole table
    int64_t slab_floats, n_red;
    int n_tasks;
    WJobs J = make_jobs(p, ws, bufs->grads, &slab_floats, &n_tasks, &n_red);
    int ta, tb;
    int64_t ra, rb;
    const WJobs JA = mlg::bjob_view(J, 3, J.n, &ta, &ra), JB = mlg::bjob_view(J, 0, 3, &tb, &rb);
    const bool fused = !rec16 && H == 64 && threads == 256;
    if (fused) {
        const int nbwd = (c.R + 3) / 4;
        hipLaunchKernelGGL((bwd4_wgrad_kernel<H>), dim3((unsigned)(nbwd + (ta + 3) / 4)), dim3(256), 0, s, c, bt, p.L,
                           ws + p.w.p_on, ws + p.w.hs, ws + p.w.gr, ws + p.w.gz, ws + p.w.gn, ws + p.w.ghn, ws + p.w.dq,
                           ws + p.w.dgi, ws + p.w.dgh, ws + p.w.msum, JA, ws + p.w.slab, nbwd);
    } else if (rec16) {
        hipLaunchKernelGGL((agent_bwd_kernel<H>), dim3(ntiles), dim3(threads), 0, s, c, bt, p.L, ws + p.w.p_on,
                           ws + p.w.hs, ws + p.w.gr, ws + p.w.gz, ws + p.w.gn, ws + p.w.ghn, ws + p.w.dq, ws + p.w.dgi,
                           ws + p.w.dgh, ws + p.w.msum);
    } else {
        hipLaunchKernelGGL((agent_bwd4_kernel<H>), dim3((c.R + 3) / 4), dim3(threads), 0, s, c, bt, p.L, ws + p.w.p_on,
                           ws + p.w.hs, ws + p.w.gr, ws + p.w.gz, ws + p.w.gn, ws + p.w.ghn, ws + p.w.dq, ws + p.w.dgi,
                           ws + p.w.dgh, ws + p.w.msum);
    }
    hipLaunchKernelGGL((agent_dx_kernel<H>), dim3(ntiles, c.T), dim3(threads), 0, s, c, ws + p.w.wihT, ws + p.w.x,
                       ws + p.w.dgi, ws + p.w.da, ws + p.w.msum);
    if (fused)
        hipLaunchKernelGGL(mlg::wgrad_block_kernel<16>, dim3((unsigned)((tb + 3) / 4)), dim3(256), 0, s, JB,
                           ws + p.w.slab);
    else
        hipLaunchKernelGGL(mlg::wgrad_block_kernel<16>, dim3((unsigned)((n_tasks + 3) / 4)), dim3(256), 0, s, J,
                           ws + p.w.slab);
    const int n_red_blocks = (int)((n_red + 255) / 256);
    hipLaunchKernelGGL(mlg::wgrad_block_reduce_kernel<16>, dim3((unsigned)n_red_blocks), dim3(256), 0, s, J,
                       ws + p.w.slab, ws + p.w.nrm);
    const int64_t n_par = p.n_agent + p.n_mixer;
    hipLaunchKernelGGL(finish_kernel, dim3((unsigned)((n_par + 1023) / 1024)), dim3(1024), 0, s, ws + p.w.part,
                       p.w.n_mix_tiles, ws + p.w.msum, bufs->params, bufs->grads, bufs->square_avg, n_par, cfg->lr,
                       cfg->optim_alpha, cfg->optim_eps, cfg->grad_norm_clip, c.N, bufs->stats, ws + p.w.nrm,
                       n_red_blocks, bufs->target_sync, bufs->trained_steps);
    return mlg::check_launch("qlearner_train");
}

}  // namespace

extern "C" int mlg_debug_set_learner_stamps(void* ptr) {
#ifdef MLG_STAMPS
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_mlg_lstamps), &ptr, sizeof(ptr));
    if (e != hipSuccess) return mlg::fail("set learner stamps: %s", hipGetErrorString(e));
    return 0;
#else
    (void)ptr;
    return mlg::fail("not a stamps build (-DMLG_STAMPS)");
#endif
}

extern "C" int64_t mlg_qlearner_param_counts(const MlgLearnerCfg* c, int64_t* n_agent, int64_t* n_mixer) {
    if (check_cfg(c)) return -1;
    Plan p = make_plan(c, c->T);
    if (n_agent) *n_agent = p.n_agent;
    if (n_mixer) *n_mixer = p.n_mixer;
    return p.n_agent + p.n_mixer;
}

extern "C" int mlg_qlearner_inline_rows(void) { return MLG_INLINE_ROWS; }

extern "C" int64_t mlg_qlearner_workspace_floats(const MlgLearnerCfg* c) {
    if (check_cfg(c)) return -1;
    Plan p = make_plan(c, c->T);
    int64_t slab, n_red;
    int tasks;
    make_jobs(p, nullptr, nullptr, &slab, &tasks, &n_red);
    return p.w.total + slab;
}

extern "C" int mlg_qlearner_train(const MlgLearnerCfg* c, const MlgLearnerBufs* b, void* stream) {
    if (check_cfg(c)) return 1;
    MLG_REQUIRE(b && b->params && b->grads && b->square_avg && b->target_params && b->workspace && b->stats,
                "qlearner_train: null buffer");
    const MlgBatch& bt = b->batch;
    MLG_REQUIRE(bt.state && bt.obs && bt.actions && bt.avail && bt.reward && bt.terminated && bt.actions_onehot && bt.filled,
                "qlearner_train: batch has null tensors");
    MLG_REQUIRE(bt.B == c->B && bt.T1 >= c->T, "qlearner_train: batch B=%d T1=%d vs cfg B=%d T=%d", bt.B, bt.T1, c->B, c->T);
    MLG_REQUIRE(!b->host_rows || c->B <= MLG_INLINE_ROWS, "qlearner_train: host_rows needs B <= %d (got %d)",
                MLG_INLINE_ROWS, c->B);
    Plan p = make_plan(c, bt.T1);
    hipStream_t s = (hipStream_t)stream;
    if (c->H == 64) return run_train<64>(p, c, b, s);
    if (c->H == 32) return run_train<32>(p, c, b, s);
    return run_train<128>(p, c, b, s);
}
