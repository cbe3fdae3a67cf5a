// gru4_device.h -- the learners' sequential GRU recurrences (forward and reverse-time backward) on 4-row tiles,
// shared by the QMIX learner (learner.hip: agent_rec4 / rec4_mixpre / agent_bwd4) and the REFIL learner
// (refil_learner.hip: rec4 / rec_bwd4). The recurrence is latency-bound (sequential in T); a 16-row tile per CU is
// MFMA-bound at 48 16x16x4 MFMAs per SIMD per step, so 4-row tiles (v_mfma_f32_4x4x1_16b_f32: 16 blocks of
// D[4x4] += A[4x1] B[1x4]) put 4x as many CUs on the T loop.
//
// Workspace layout (t-major, both learners): GI [T][R][3H] with the gate biases folded ([b_ir + b_hr + W_ir x |
// b_iz + b_hz + W_iz x | b_in + W_in x]), HS [T+1][R][H] (HS[0] = 0), gates r / z / n / (W_hn h + b_hn) [T][R][H],
// dGI / dGH [T][R][3H]. Restates nn.GRUCell (drqn_agent.py:33, entity_rnn_agent.py:63) and its autograd.
#pragma once
#include <hip/hip_runtime.h>

#include "mlg_device.h"

// prefetch depth (steps) of the recurrences' per-step operand rings (even: the LDS double buffer alternates)
#ifndef MLG_REC_PD
#define MLG_REC_PD 4
#endif
#ifndef MLG_BWD_PD
#define MLG_BWD_PD 4
#endif

constexpr int MLG_BWD_MAXA = 96;  // output-layer rows staged in LDS by the backward recurrences (host-checked)

namespace mlg {

struct NoStamps {  // the recurrences' diagnostic stamp hooks, compiled out
    unsigned long long steps;
    __device__ void init() {}
    __device__ void mark(int) {}
    __device__ void flush(int) {}
};

struct Gru4Fwd {
    int R;                         // rows of this net
    const float* whh;              // W_hh [3H][H]
    const float* bhh;              // b_hh [3H]
    const float* gi;               // GI [T][R][3H]
    float* hs;                     // HS [T+1][R][H]
    float *gr, *gz, *gn, *ghn;     // gates [T][R][H] (stored when `gates`)
    bool gates;                    // online net: the backward needs the gates
};

// One 4-row tile of the forward recurrence over Te steps. Wave w owns hidden features 16w..16w+15: block b = 4g + fg
// computes gate g (r, z, W_hn h; g = 3 idle) of features 16w + 4fg + i for the tile's 4 rows, W_hh rows of the
// block in VGPRs (H per lane). A row / register transpose across the wave's four 16-lane rows (rows_transpose4,
// four VALU lane swaps) then gives every lane the three gates of one (feature 16w + 4fg + g, row): all 64 lanes
// finish one GRU cell each. H/16 waves.
template <int H, class ST>
__device__ __forceinline__ void gru4_fwd(const Gru4Fwd& a, int tile, int Te, ST& lst) {
    constexpr int LDA = H + 4;
    __shared__ __attribute__((aligned(16))) float hs[2][4 * LDA];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int b = lane >> 2, q = lane & 3;  // block, and i (A / D register) or j (B / D column = row)
    const int g = b >> 2, fg = b & 3;
    const int R = a.R;
    const int r = tile * 4 + q;  // this lane's row as a B / D column
    const bool valid = r < R;
    const int rr = valid ? r : 0;
    const int fA = 16 * w + 4 * fg + q;  // A operand: feature row of W_hh for this lane (i = q)
    const int fD = 16 * w + 4 * fg;      // D: features fD..fD+3 of gate g at row r
    const int f = fD + g;                // after the transpose: the lane's cell is (feature f, row r)
    float wa[H];
#pragma unroll
    for (int k4 = 0; k4 < H / 4; ++k4) {
        const floatx4 v = g < 3 ? ld4(a.whh + (int64_t)(g * H + fA) * H + 4 * k4) : floatx4{0.f, 0.f, 0.f, 0.f};
        wa[4 * k4] = v.x;
        wa[4 * k4 + 1] = v.y;
        wa[4 * k4 + 2] = v.z;
        wa[4 * k4 + 3] = v.w;
    }
    const floatx4 bhn = ld4(a.bhh + 2 * H + fD);
    for (int i = tid; i < 4 * LDA; i += blockDim.x) hs[0][i] = 0.f;
    const __amdgpu_buffer_rsrc_t rs_gi = mlg_rsrc(a.gi), rs_h = mlg_rsrc(a.hs), rs_r = mlg_rsrc(a.gr),
                                 rs_z = mlg_rsrc(a.gz), rs_n = mlg_rsrc(a.gn), rs_hn = mlg_rsrc(a.ghn);
    st1_rs(rs_h, valid ? (rr * H + f) * 4 : (int)0x80000000u, 0, 0.f);  // HS[0]
    // per-step inputs: the MFMA init of rows 0 / 1 (GI r / z part of features fD..) and the lane's GI n element
    const int gq = g == 1 ? 1 : 0;
    const int vo_gp = (rr * 3 * H + gq * H + fD) * 4, vo_gn = (rr * 3 * H + 2 * H + f) * 4;
    struct In {
        floatx4 gp;
        float gn;
    };
    auto load_in = [&](int t, In& d) {
        const int so = t * R * 3 * H * 4;
        d.gp = ld4_rs(rs_gi, vo_gp, so);
        d.gn = ld1_rs(rs_gi, vo_gn, so);
    };
    const int vo_st = valid ? (rr * H + f) * 4 : (int)0x80000000u;
    const bool online = a.gates;
    float hprev = 0.f;  // h_{t-1} of the lane's cell: its own previous output
    auto step = [&](int t, const In& in, int cur) {
        const float* hrow = hs[cur] + q * LDA;
        floatx4 hv[H / 4];  // the whole h row first: the MFMA chain then never waits on LDS
#pragma unroll
        for (int k4 = 0; k4 < H / 4; ++k4) hv[k4] = ld4(hrow + 4 * k4);
        // two accumulation chains (even / odd k quads) halve the dependent-MFMA latency; summed at the end
        floatx4 acc0 = g == 2 ? bhn : (g == 3 ? floatx4{0.f, 0.f, 0.f, 0.f} : in.gp), acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k4 = 0; k4 < H / 4; k4 += 2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(wa[4 * k4 + e], hv[k4][e], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_4x4x1f32(wa[4 * k4 + 4 + e], hv[k4 + 1][e], acc1, 0, 0, 0);
            }
        }
        const floatx4 acc = acc0 + acc1;
        float ar = acc[0], az = acc[1], ahn = acc[2], a3 = acc[3];
        rows_transpose4(ar, az, ahn, a3);  // gate g of (feature f, row r) now in register g
        lst.mark(0);
        const float rg = fast_sigmoid(ar), zg = fast_sigmoid(az);
        const float ng = fast_tanh(in.gn + rg * ahn);
        const float hn = ng + zg * (hprev - ng);
        hs[cur ^ 1][q * LDA + f] = hn;
        hprev = hn;
        lst.mark(2);
        const int vo = t < Te ? vo_st : (int)0x80000000u;  // t >= Te: padding step (see below)
        const int vg = online ? vo : (int)0x80000000u;
        const int so = (t < Te ? t : 0) * R * H * 4;
        st1_rs(rs_h, vo, so + R * H * 4, hn);  // HS[t + 1]
        st1_rs(rs_r, vg, so, rg);
        st1_rs(rs_z, vg, so, zg);
        st1_rs(rs_n, vg, so, ng);
        st1_rs(rs_hn, vg, so, ahn);
        lst.mark(3);
        __syncthreads();
        lst.mark(4);
        ++lst.steps;
    };
    // GI rows are prefetched MLG_REC_PD steps ahead (clamped, unconditional loads) into a register ring. The step
    // count is padded to a multiple of MLG_REC_PD (padding steps store nothing): no control flow inside the
    // unrolled body, so every ring slot keeps its registers and the loads are waited for only where consumed.
    In ring[MLG_REC_PD];
#pragma unroll
    for (int i = 0; i < MLG_REC_PD; ++i) load_in(i < Te ? i : Te - 1, ring[i]);
    __syncthreads();
    lst.mark(5);
    for (int t0 = 0; t0 < Te; t0 += MLG_REC_PD) {
#pragma unroll
        for (int i = 0; i < MLG_REC_PD; ++i) {
            const int t = t0 + i;
            step(t, ring[i], i & 1);
            // refill the slot only once the step has consumed it: the load then targets the slot's own registers
            // (no register rotation at the loop back-edge, which would wait for every load in flight)
            load_in(t + MLG_REC_PD < Te ? t + MLG_REC_PD : Te - 1, ring[i]);
            lst.mark(1);
        }
    }
}

struct Gru4Bwd {
    int R;                         // rows (online net)
    int T;                         // steps of the batch: dQ / actions exist for t < T - 1
    int A, N;                      // actions; agents per episode (action row stride)
    const float* whh;              // W_hh [3H][H]
    const float* wq;               // output layer [A][H] (dh += dQ W_q[a])
    const float *hs, *gr, *gz, *gn, *ghn;
    const float* dq;               // dQ of the chosen action [T - 1][R]
    const int64_t* actions;        // the batch's actions; row's action at abase + t N (int64 elements)
    float *dgi, *dgh;              // [T][R][3H]
};

// One 4-row tile of the reverse-time backward over Te steps (rows past Te zeroed: they are wgrad rows). Wave w owns
// hidden features 16w..16w+15; block b = 4kq + fg accumulates W_hh^T dGH for features 16w + 4fg + i over the K
// quarter kq (48 of the 3H gate rows, W_hh columns in VGPRs). The four quarter partials are summed across the wave's
// 16-lane rows with a transposing reduction (rows_sum_transpose4): lane (row kq, fg, j) ends up owning feature
// 16w + 4fg + kq of row j, so all 64 lanes run the elementwise GRU backward, one (feature, row) each. abase: the
// int64 element offset of this lane's row's actions at t = 0. H/16 waves.
template <int H, class ST>
__device__ __forceinline__ void gru4_bwd(const Gru4Bwd& a, int tile, int Te, int64_t abase, ST& lst) {
    constexpr int LDG = 3 * H + 4;
    constexpr int KQ = 3 * H / 4;  // gate rows per K quarter
    __shared__ __attribute__((aligned(16))) float sgh[2][4 * LDG];
    __shared__ __attribute__((aligned(16))) float w2s[MLG_BWD_MAXA * H];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int blk = lane >> 2, q = lane & 3, kq = blk >> 2, fg = blk & 3;
    const int r = tile * 4 + q;
    const bool valid = r < a.R;
    const int R = a.R, N = a.N;
    const int fD = 16 * w + 4 * fg;
    const int f = fD + kq;  // the lane's (feature, row) after the reduction
    const int rr = valid ? r : 0;
    struct Raw {  // per-step operands as stored by the forward, for (feature f, row r)
        float rg, zg, ng, ghn, hp, dq;
        int a;
    };
    // Buffer loads: the lane part of every offset is fixed, the step part is a wave-uniform SGPR offset, so a
    // step's loads cost no VALU address arithmetic.
    const __amdgpu_buffer_rsrc_t rs_r = mlg_rsrc(a.gr), rs_z = mlg_rsrc(a.gz), rs_n = mlg_rsrc(a.gn),
                                 rs_hn = mlg_rsrc(a.ghn), rs_hs = mlg_rsrc(a.hs), rs_dq = mlg_rsrc(a.dq),
                                 rs_act = mlg_rsrc(reinterpret_cast<const float*>(a.actions));
    const int vo_g = (rr * H + f) * 4, vo_dq = rr * 4, vo_act = (int)(abase * 8);
    auto load_raw = [&](int t, Raw& s) {
        const int so = t * R * H * 4;
        s.rg = ld1_rs(rs_r, vo_g, so);
        s.zg = ld1_rs(rs_z, vo_g, so);
        s.ng = ld1_rs(rs_n, vo_g, so);
        s.ghn = ld1_rs(rs_hn, vo_g, so);
        s.hp = ld1_rs(rs_hs, vo_g, so);  // HS[t] = h_{t-1}
        const int tq = t < a.T - 1 ? t : a.T - 2;
        s.dq = ld1_rs(rs_dq, vo_dq, tq * R * 4);
        // 32-bit load of the action's low word (little-endian int64), unconditional: no branch around it, and no
        // dead high half whose pending load would block the reuse of its register
        const int act = __float_as_int(ld1_rs(rs_act, vo_act, tq * N * 8));
        s.a = t < a.T - 1 ? act : -1;
    };
    // the first steps' operands are requested before anything else is queued on the vector memory path
    Raw ring[MLG_BWD_PD];
#pragma unroll
    for (int i = 0; i < MLG_BWD_PD; ++i) load_raw(Te - 1 - i > 0 ? Te - 1 - i : 0, ring[i]);
    float wt[KQ];  // A operand: W_hh[kq * KQ + kk][fD + i] (i = q)
#pragma unroll
    for (int kk = 0; kk < KQ; ++kk) wt[kk] = a.whh[(int64_t)(kq * KQ + kk) * H + fD + q];
    {  // output rows for dh += dq W_q[a], staged in LDS: a thread's loads all issued before its first LDS write (the
       // strided copy loop waited for each load in turn, ahead of the first step)
        constexpr int PER = 8;
        const int n = a.A * H, nt = blockDim.x;
        for (int i0 = tid; i0 < n; i0 += PER * nt) {
            float v[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) v[u] = i0 + u * nt < n ? a.wq[i0 + u * nt] : 0.f;
#pragma unroll
            for (int u = 0; u < PER; ++u)
                if (i0 + u * nt < n) w2s[i0 + u * nt] = v[u];
        }
    }
    {  // steps past max_t_filled: zero deltas (wgrad rows); the tile's rows are contiguous per step
        const int nv = min(4, R - tile * 4) * 3 * H / 4;  // float4s per step and array
        for (int t = Te; t < a.T; ++t) {
            float* zi = a.dgi + ((int64_t)t * R + tile * 4) * 3 * H;
            float* zh = a.dgh + ((int64_t)t * R + tile * 4) * 3 * H;
            for (int i = tid; i < nv; i += blockDim.x) {
                reinterpret_cast<floatx4*>(zi)[i] = floatx4{0.f, 0.f, 0.f, 0.f};
                reinterpret_cast<floatx4*>(zh)[i] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
        }
    }
    // Every gate delta is dh times a factor of the saved activations (the GRU backward is linear in dh), and the
    // output-layer term dq W_q[a] does not depend on dh either: both are formed one step ahead, off the dh -> dh chain.
    struct Coef {
        float cr, cz, cn, chn, ch, dw;
    };
    auto coef = [&](const Raw& s, Coef& k) {
        const bool take = valid && s.a >= 0;
        const float w2 = w2s[(take ? s.a : 0) * H + f];
        const float cn = (1.f - s.zg) * (1.f - s.ng * s.ng);  // dn' = dh (1 - z)(1 - n^2)
        k.cn = cn;
        k.cr = cn * s.ghn * (s.rg * (1.f - s.rg));      // dr' = dn' (W_hn h + b_hn) r (1 - r)
        k.cz = (s.hp - s.ng) * (s.zg * (1.f - s.zg));  // dz' = dh (h_{t-1} - n) z (1 - z)
        k.chn = cn * s.rg;                              // d(W_hn h + b_hn) = dn' r
        k.ch = s.zg;                                    // direct path dh_{t-1} += dh z
        k.dw = (take ? s.dq : 0.f) * w2;
    };
    float dh = 0.f;
    const __amdgpu_buffer_rsrc_t rs_gi = mlg_rsrc(a.dgi), rs_gh = mlg_rsrc(a.dgh);
    const int vo_st = valid ? (r * 3 * H + f) * 4 : (int)0x80000000u;
    auto step = [&](int t, const Coef& k, int cur) {
        dh += k.dw;
        const float drp = dh * k.cr, dzp = dh * k.cz, dnp = dh * k.cn, dghn = dh * k.chn, dhd = dh * k.ch;
        float* gh = sgh[cur] + q * LDG + f;
        gh[0] = drp;
        gh[H] = dzp;
        gh[2 * H] = dghn;
        lst.mark(2);
        __syncthreads();
        lst.mark(4);
        const float* ghr = sgh[cur] + q * LDG + kq * KQ;
        floatx4 gv[KQ / 4];
#pragma unroll
        for (int k4 = 0; k4 < KQ / 4; ++k4) gv[k4] = ld4(ghr + 4 * k4);
        // the step's global stores go out behind the barrier, in the shadow of the MFMA chain
        const int vo = t >= 0 ? vo_st : (int)0x80000000u;  // t < 0: padding step, every lane dropped
        const int so = (t >= 0 ? t : 0) * R * 3 * H * 4;
        st1_rs(rs_gi, vo, so, drp);
        st1_rs(rs_gi, vo, so + H * 4, dzp);
        st1_rs(rs_gi, vo, so + 2 * H * 4, dnp);
        st1_rs(rs_gh, vo, so, drp);
        st1_rs(rs_gh, vo, so + H * 4, dzp);
        st1_rs(rs_gh, vo, so + 2 * H * 4, dghn);
        lst.mark(3);
        floatx4 p0 = {0.f, 0.f, 0.f, 0.f}, p1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k4 = 0; k4 < KQ / 4; k4 += 2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                p0 = __builtin_amdgcn_mfma_f32_4x4x1f32(wt[4 * k4 + e], gv[k4][e], p0, 0, 0, 0);
                p1 = __builtin_amdgcn_mfma_f32_4x4x1f32(wt[4 * k4 + 4 + e], gv[k4 + 1][e], p1, 0, 0, 0);
            }
        }
        const floatx4 part = p0 + p1;
        dh = dhd + rows_sum_transpose4(part[0], part[1], part[2], part[3]);  // (q0 + q1) + (q2 + q3)
        lst.mark(0);
        ++lst.steps;
    };
    __syncthreads();  // w2s staged
    Coef kc;
    coef(ring[0], kc);
    lst.mark(5);
    // step count padded to a multiple of MLG_BWD_PD (padding steps t < 0 store nothing; see gru4_fwd)
    for (int t0 = Te - 1; t0 >= 0; t0 -= MLG_BWD_PD) {
#pragma unroll
        for (int i = 0; i < MLG_BWD_PD; ++i) {
            const int t = t0 - i;
            load_raw(t - MLG_BWD_PD > 0 ? t - MLG_BWD_PD : 0, ring[i]);  // slot i (step t) is consumed
            Coef kn;
            coef(ring[(i + 1) % MLG_BWD_PD], kn);  // step t - 1
            lst.mark(1);
            step(t, kc, i & 1);
            kc = kn;
        }
    }
}

}  // namespace mlg
