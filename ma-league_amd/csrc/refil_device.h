// refil_device.h -- REFIL (config 5) building blocks for gfx950, shared by the rollout and the learner:
//
//   * wave-level f32 MFMA (16x16x4) GEMMs over one 16-row tile: rows = entities (fc1, in_trans) or
//     agent rows of two items (out_trans, fc2, GRU, fc3); weights [M][K] row-major from HBM/L2, activations
//     from LDS (row-major) or from registers (the D layout of the previous GEMM, see mlg_device.h)
//   * EntityAttentionLayer forward / backward for one item (src/marl/modules/layers/attention.py:24-79):
//     lane = (head, query), 4 heads x 16 query slots, keys in LDS; -inf pre-mask, softmax, NaN rows -> 0
//   * the entity env variant (oracle/env_ref.c envref_reset_entity / envref_entities)
//
// Sizes fixed by the kernels (host-checked): n_entities <= 16 (one MFMA tile), n_agents <= 8 (two items per
// agent-row tile), attn_embed_dim = rnn_hidden_dim = hypernet_embed = 64, attn_n_heads = 4 (head_dim 16),
// mixing_embed_dim = 32, entity input dim ED + A <= 48.
#pragma once
#include "agent_device.h"

namespace refil {

constexpr int NE = 16;            // entity slots per item
constexpr int NAS = 8;            // agent-row slots per item
constexpr int EMB = 64;           // attention / hidden width
constexpr int NH = 4, HD = 16;    // heads, head dim
constexpr int EM = 32;            // mixing_embed_dim
constexpr int LDX = EMB + 4;      // LDS row stride of 64-wide activations (conflict-free 16-row reads)
constexpr int LDQ = 3 * EMB + 4;  // qkv rows
constexpr int KMAX = 48;          // entity input width, padded
constexpr int LDI = KMAX + 4;

// wave-local barrier: orders the LDS writes of some lanes before the reads of others (single wave)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- packed weight blocks ---------------------------------------------------------------------------
// Agent (EntityAttentionRNNAgent, entity_rnn_agent.py:9-26): K1 = entity input width padded to 16.
//   w1 [64][K1], b1 [64], win [192][64], wout [64][64], bout [64], w2 [64][64], b2 [64],
//   wih [192][64], whh [192][64], bih [192], bhh [192], brz [128] (= b_ih + b_hh of r, z), w3 [Ap][64], b3 [Ap]
// Canonical flat order (named_parameters): fc1.w [64][D0], fc1.b, attn.in_trans.w [192][64], attn.out_trans.w,
//   attn.out_trans.b, fc2.w, fc2.b, rnn.weight_ih, rnn.weight_hh, rnn.bias_ih, rnn.bias_hh, fc3.w [A][64], fc3.b [A]
// gsp section: W_ih / W_hh as split-bf16 MFMA A operands, [mat 2][mt 4][gate 3][kk 2][piece 3][lane 64] x 16 B
constexpr int64_t REFIL_GSP = 2 * 4 * 3 * 2 * 3 * 64 * 4;
// wsp section: in_trans [192][64] (tiles 0-11), out_trans [64][64] (12-15), fc2 [64][64] (16-19), fc1 [64][D0]
// (20-23, K slots >= D0 zero) and fc3 [A][64] (24-25, rows >= A zero) as split-bf16 MFMA A operands,
// [tile 26][kk 2][piece 3][lane 64] x 16 B
constexpr int REFIL_WSP_WOUT = 12, REFIL_WSP_W2 = 16, REFIL_WSP_W1 = 20, REFIL_WSP_W3 = 24;
constexpr int64_t REFIL_WSP = 26 * 2 * 3 * 64 * 4;

struct RAgent {
    int D0, K1, A, Ap;
    int64_t w1, b1, win, wout, bout, w2, b2, wih, whh, bih, bhh, brz, w3, b3, gsp, wsp, total;
    // canonical offsets
    int64_t c_w1, c_b1, c_win, c_wout, c_bout, c_w2, c_b2, c_wih, c_whh, c_bih, c_bhh, c_w3, c_b3, c_total;
};

__host__ __device__ inline RAgent make_ragent(int D0, int A) {
    RAgent L;
    L.D0 = D0;
    L.K1 = (D0 + 15) / 16 * 16;
    L.A = A;
    L.Ap = (A + 15) / 16 * 16;
    int64_t o = 0;
    auto take = [&](int64_t n) { int64_t r = o; o += mlg_align4(n); return r; };
    L.w1 = take((int64_t)EMB * L.K1);
    L.b1 = take(EMB);
    L.win = take(3 * EMB * EMB);
    L.wout = take(EMB * EMB);
    L.bout = take(EMB);
    L.w2 = take(EMB * EMB);
    L.b2 = take(EMB);
    L.wih = take(3 * EMB * EMB);
    L.whh = take(3 * EMB * EMB);
    L.bih = take(3 * EMB);
    L.bhh = take(3 * EMB);
    L.brz = take(2 * EMB);
    L.w3 = take((int64_t)L.Ap * EMB);
    L.b3 = take(L.Ap);
    L.gsp = take(REFIL_GSP);  // rollout GRU weights pre-split (gru_tile_b16 layout), written by mlg_refil_pack_agent
    L.wsp = take(REFIL_WSP);  // rollout in_trans / out_trans / fc2 weights pre-split, written by mlg_refil_pack_agent
    L.total = o;
    int64_t c = 0;
    L.c_w1 = c; c += (int64_t)EMB * D0;
    L.c_b1 = c; c += EMB;
    L.c_win = c; c += 3 * EMB * EMB;
    L.c_wout = c; c += EMB * EMB;
    L.c_bout = c; c += EMB;
    L.c_w2 = c; c += EMB * EMB;
    L.c_b2 = c; c += EMB;
    L.c_wih = c; c += 3 * EMB * EMB;
    L.c_whh = c; c += 3 * EMB * EMB;
    L.c_bih = c; c += 3 * EMB;
    L.c_bhh = c; c += 3 * EMB;
    L.c_w3 = c; c += (int64_t)A * EMB;
    L.c_b3 = c; c += A;
    L.c_total = c;
    return L;
}

// Attention hypernet (AttentionHyperNet, flex_qmix.py:5-53) with mixing_embed_dim outputs:
//   w1 [64][K1], b1 [64], win [192][64], wout [64][64], bout [64], w2 [32][64], b2 [32]
// canonical (named_parameters): fc1.w [64][D0], fc1.b, attn.in_trans.w, attn.out_trans.w, attn.out_trans.b,
//   fc2.w [32][64], fc2.b [32].  FlexQMixer = hyper_w_1, hyper_w_final, hyper_b_1, V (flex_qmix.py:61-66).
struct RHyper {
    int D0, K1;
    int64_t w1, b1, win, wout, bout, w2, b2, total;
    int64_t c_w1, c_b1, c_win, c_wout, c_bout, c_w2, c_b2, c_total;
};

__host__ __device__ inline RHyper make_rhyper(int D0) {
    RHyper L;
    L.D0 = D0;
    L.K1 = (D0 + 15) / 16 * 16;
    int64_t o = 0;
    auto take = [&](int64_t n) { int64_t r = o; o += mlg_align4(n); return r; };
    L.w1 = take((int64_t)EMB * L.K1);
    L.b1 = take(EMB);
    L.win = take(3 * EMB * EMB);
    L.wout = take(EMB * EMB);
    L.bout = take(EMB);
    L.w2 = take(EM * EMB);
    L.b2 = take(EM);
    L.total = o;
    int64_t c = 0;
    L.c_w1 = c; c += (int64_t)EMB * D0;
    L.c_b1 = c; c += EMB;
    L.c_win = c; c += 3 * EMB * EMB;
    L.c_wout = c; c += EMB * EMB;
    L.c_bout = c; c += EMB;
    L.c_w2 = c; c += EM * EMB;
    L.c_b2 = c; c += EM;
    L.c_total = c;
    return L;
}

// ---- wave GEMM helpers ---------------------------------------------------------------------------------
// acc[i] (D layout: lane (col, g), reg r = output feature (mt0 + i) * 16 + 4g + r of tile row col)
//   += W[(mt0 + i) * 16 + col][k] * X[col][k]   over k < 16 * kchunks
template <int MT>
__device__ __forceinline__ void bias_init(floatx4 (&acc)[MT], const float* bias, int mt0, int lane) {
    const int g = lane >> 4;
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[i] = bias ? ld4(bias + (mt0 + i) * 16 + 4 * g) : floatx4{0.f, 0.f, 0.f, 0.f};
}

template <int MT>
__device__ __forceinline__ void mm_lds(floatx4 (&acc)[MT], const float* __restrict__ W, int ldw, int mt0, const float* X,
                                       int ldx, int kchunks, int lane) {
    const int col = lane & 15, g = lane >> 4;
    const float* xr = X + col * ldx + 4 * g;
    const float* wr = W + (int64_t)(mt0 * 16 + col) * ldw + 4 * g;
    for (int kc = 0; kc < kchunks; ++kc) {
        const floatx4 xv = ld4(xr + kc * 16);
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i] = mfma_chunk(ld4(wr + (int64_t)i * 16 * ldw + kc * 16), xv, acc[i]);
    }
}

template <int MT, int KC>
__device__ __forceinline__ void mm_reg(floatx4 (&acc)[MT], const float* __restrict__ W, int ldw, int mt0,
                                       const floatx4 (&x)[KC], int lane) {
    const int col = lane & 15, g = lane >> 4;
    const float* wr = W + (int64_t)(mt0 * 16 + col) * ldw + 4 * g;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i] = mfma_chunk(ld4(wr + (int64_t)i * 16 * ldw + kc * 16), x[kc], acc[i]);
}

// same with a per-lane row pointer (rows scattered in HBM): lane (col, g) passes the base of its tile row col
template <int MT>
__device__ __forceinline__ void mm_ptr(floatx4 (&acc)[MT], const float* __restrict__ W, int ldw, int mt0, const float* xrow,
                                       int kchunks, int lane) {
    const int col = lane & 15, g = lane >> 4;
    const float* xr = xrow + 4 * g;
    const float* wr = W + (int64_t)(mt0 * 16 + col) * ldw + 4 * g;
    for (int kc = 0; kc < kchunks; ++kc) {
        const floatx4 xv = ld4(xr + kc * 16);
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i] = mfma_chunk(ld4(wr + (int64_t)i * 16 * ldw + kc * 16), xv, acc[i]);
    }
}

__device__ __forceinline__ void st_row(float* Y, int ldy, int mt, const floatx4 v, int lane) {
    *reinterpret_cast<floatx4*>(Y + (lane & 15) * ldy + mt * 16 + 4 * (lane >> 4)) = v;
}

__device__ __forceinline__ floatx4 relu4(floatx4 v) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
    return v;
}

// Y[16][64 * G] rows of LDS = act(bias + W X) for 4*G output tiles (G groups of 4 tiles)
template <bool RELU>
__device__ __forceinline__ void dense_lds(const float* __restrict__ W, int ldw, const float* bias, int mtiles,
                                          const float* X, int ldx, int kchunks, float* Y, int ldy, int lane) {
    for (int m0 = 0; m0 < mtiles; m0 += 4) {
        floatx4 acc[4];
        bias_init<4>(acc, bias, m0, lane);
        mm_lds<4>(acc, W, ldw, m0, X, ldx, kchunks, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) st_row(Y, ldy, m0 + i, RELU ? relu4(acc[i]) : acc[i], lane);
    }
}

// ---- EntityAttentionLayer core for one item ---------------------------------------------------------
// qkv: LDS [NE][LDQ] (query cols 0..63, key 64..127, value 128..191; chunk(3) of in_trans, attention.py:33);
// mrow[q]: pre-mask bits of query row q (bit j = entity j masked); nq <= 16 queries; keys k >= ne are masked.
// Lane (h = lane >> 4, q = lane & 15). Output o row q (cols h*16..) in LDS; P[h][q][k] saved when non-null
// (global or LDS, row stride 16). Rows with every key masked: softmax NaN -> 0 (attention.py:59).
// General form: query rows at qb (row stride ldq), key / value rows at kb / vb (row stride ldkv).
__device__ inline void attn_fwd_split(const float* qb, int ldq, const float* kb, const float* vb, int ldkv,
                                      const uint32_t* mrow, int nq, int ne, float* o, int ldo, float* P, int lane) {
    const int h = lane >> 4, q = lane & 15;
    if (q >= nq) return;
    float qv[HD];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const floatx4 v = ld4(qb + q * ldq + h * HD + 4 * c);
        qv[4 * c] = v[0]; qv[4 * c + 1] = v[1]; qv[4 * c + 2] = v[2]; qv[4 * c + 3] = v[3];
    }
    const uint32_t m = mrow[q] | (ne < 32 ? (~0u << ne) : 0u);
    float s[NE];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const float* kr = kb + k * ldkv + h * HD;
        float d = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const floatx4 kv = ld4(kr + 4 * c);
            d = fmaf(qv[4 * c], kv[0], d);
            d = fmaf(qv[4 * c + 1], kv[1], d);
            d = fmaf(qv[4 * c + 2], kv[2], d);
            d = fmaf(qv[4 * c + 3], kv[3], d);
        }
        s[k] = ((m >> k) & 1u) ? -INFINITY : d * 0.25f;  // / sqrt(head_dim) = / 4 (exact)
        mx = fmaxf(mx, s[k]);
    }
    float ov[HD];
#pragma unroll
    for (int d = 0; d < HD; ++d) ov[d] = 0.f;
    if (mx != -INFINITY) {
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            s[k] = ((m >> k) & 1u) ? 0.f : expf(s[k] - mx);
            sum += s[k];
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) s[k] = s[k] / sum;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const float* vr = vb + k * ldkv + h * HD;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const floatx4 vv = ld4(vr + 4 * c);
                ov[4 * c] = fmaf(s[k], vv[0], ov[4 * c]);
                ov[4 * c + 1] = fmaf(s[k], vv[1], ov[4 * c + 1]);
                ov[4 * c + 2] = fmaf(s[k], vv[2], ov[4 * c + 2]);
                ov[4 * c + 3] = fmaf(s[k], vv[3], ov[4 * c + 3]);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NE; ++k) s[k] = 0.f;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
        *reinterpret_cast<floatx4*>(o + q * ldo + h * HD + 4 * c) = floatx4{ov[4 * c], ov[4 * c + 1], ov[4 * c + 2], ov[4 * c + 3]};
    if (P) {
        float* pr = P + (h * 16 + q) * NE;
#pragma unroll
        for (int c = 0; c < 4; ++c)
            *reinterpret_cast<floatx4*>(pr + 4 * c) = floatx4{s[4 * c], s[4 * c + 1], s[4 * c + 2], s[4 * c + 3]};
    }
}

__device__ inline void attn_fwd(const float* qkv, const uint32_t* mrow, int nq, int ne, float* o, int ldo, float* P,
                                int lane) {
    attn_fwd_split(qkv, LDQ, qkv + EMB, qkv + 2 * EMB, LDQ, mrow, nq, ne, o, ldo, P, lane);
}


// attn_fwd_split for nq <= 8 using all 64 lanes: lane (h = lane >> 4, q = lane & 7, half = (lane >> 3) & 1) scores
// keys [8 half, 8 half + 8); max, sum and the weighted values are combined with the partner lane (lane ^ 8 = DPP
// row_ror:8 inside the 16-lane row, a VALU move instead of an LDS permute). Rollout form (the recorded actions are
// the fp32 oracle's argmax within the parity tests' 1e-4 Q tolerance): softmax on v_exp_f32 (__expf) and one
// reciprocal per row, exp(s - max) * (1 / sum).
__device__ __forceinline__ float xor8f(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, true));
}
__device__ inline void attn_fwd_half(const float* qb, int ldq, const float* kb, const float* vb, int ldkv,
                                     const uint32_t* mrow, int nq, int ne, float* o, int ldo, int lane) {
    const int h = lane >> 4, q = lane & 7, half = (lane >> 3) & 1, k0 = half * 8;
    const bool qv_ok = q < nq;
    float qv[HD];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const floatx4 v = ld4(qb + q * ldq + h * HD + 4 * c);
        qv[4 * c] = v[0]; qv[4 * c + 1] = v[1]; qv[4 * c + 2] = v[2]; qv[4 * c + 3] = v[3];
    }
    const uint32_t m = (qv_ok ? mrow[q] : 0xFFFFFFFFu) | (ne < 32 ? (~0u << ne) : 0u);
    float s[8];
    float mx = -INFINITY;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
        const int k = k0 + kk;
        const float* kr = kb + k * ldkv + h * HD;
        float d = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const floatx4 kv = ld4(kr + 4 * c);
            d = fmaf(qv[4 * c], kv[0], d);
            d = fmaf(qv[4 * c + 1], kv[1], d);
            d = fmaf(qv[4 * c + 2], kv[2], d);
            d = fmaf(qv[4 * c + 3], kv[3], d);
        }
        s[kk] = ((m >> k) & 1u) ? -INFINITY : d * 0.25f;
        mx = fmaxf(mx, s[kk]);
    }
    mx = fmaxf(mx, xor8f(mx));
    float ov[HD];
#pragma unroll
    for (int d = 0; d < HD; ++d) ov[d] = 0.f;
    float sum = 0.f;
    if (mx != -INFINITY) {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            s[kk] = ((m >> (k0 + kk)) & 1u) ? 0.f : __expf(s[kk] - mx);
            sum += s[kk];
        }
    }
    sum += xor8f(sum);
    if (mx != -INFINITY) {
        const float inv = 1.f / sum;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            const float p = s[kk] * inv;
            const float* vr = vb + (k0 + kk) * ldkv + h * HD;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const floatx4 vv = ld4(vr + 4 * c);
                ov[4 * c] = fmaf(p, vv[0], ov[4 * c]);
                ov[4 * c + 1] = fmaf(p, vv[1], ov[4 * c + 1]);
                ov[4 * c + 2] = fmaf(p, vv[2], ov[4 * c + 2]);
                ov[4 * c + 3] = fmaf(p, vv[3], ov[4 * c + 3]);
            }
        }
    }
#pragma unroll
    for (int d = 0; d < HD; ++d) ov[d] += xor8f(ov[d]);
    if (qv_ok && half == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
            *reinterpret_cast<floatx4*>(o + q * ldo + h * HD + 4 * c) =
                floatx4{ov[4 * c], ov[4 * c + 1], ov[4 * c + 2], ov[4 * c + 3]};
    }
}

// Backward of attn_fwd for one item. P: [NH][16][16] saved weights; dO: rows q < nq (cols h*16..);
// DS: LDS scratch [NH][16][16]; dqkv: LDS [NE][LDQ], written (ACC = false) or accumulated (ACC = true):
// dQ rows < nq (rows >= nq get 0 when writing), dK / dV all 16 rows.
//   dP = dO V^T, dS = P (dP - sum_k P dP) / 4, dQ = dS K, dK = dS^T Q, dV = P^T dO
// (masked keys and fully masked rows have P = 0 -> dS = 0, matching the masked_fill backward)
// force-inlined: a call takes generic pointers, so every access became FLAT (LDS operands included: their waits
// then also wait for the vector memory path); inlined, the LDS operands are ds_ reads and P a global load
template <bool ACC>
__device__ __forceinline__ void attn_bwd(const float* qkv, const float* P, int nq, const float* dO, int ldo, float* DS,
                                         float* dqkv,
                                int lane) {
    const int h = lane >> 4, q = lane & 15;
    {
        float dq[HD];
#pragma unroll
        for (int d = 0; d < HD; ++d) dq[d] = 0.f;
        float ds[NE];
        if (q < nq) {
            float dov[HD];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const floatx4 v = ld4(dO + q * ldo + h * HD + 4 * c);
                dov[4 * c] = v[0]; dov[4 * c + 1] = v[1]; dov[4 * c + 2] = v[2]; dov[4 * c + 3] = v[3];
            }
            const float* pr = P + (h * 16 + q) * NE;
            float sdp = 0.f;
#pragma unroll
            for (int k = 0; k < NE; ++k) {
                const float* vr = qkv + k * LDQ + 2 * EMB + h * HD;
                float d = 0.f;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const floatx4 vv = ld4(vr + 4 * c);
                    d = fmaf(dov[4 * c], vv[0], d);
                    d = fmaf(dov[4 * c + 1], vv[1], d);
                    d = fmaf(dov[4 * c + 2], vv[2], d);
                    d = fmaf(dov[4 * c + 3], vv[3], d);
                }
                ds[k] = d;
                sdp = fmaf(pr[k], d, sdp);
            }
#pragma unroll
            for (int k = 0; k < NE; ++k) {
                const float p = pr[k];
                ds[k] = p * (ds[k] - sdp) * 0.25f;
                const float* kr = qkv + k * LDQ + EMB + h * HD;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const floatx4 kv = ld4(kr + 4 * c);
                    dq[4 * c] = fmaf(ds[k], kv[0], dq[4 * c]);
                    dq[4 * c + 1] = fmaf(ds[k], kv[1], dq[4 * c + 1]);
                    dq[4 * c + 2] = fmaf(ds[k], kv[2], dq[4 * c + 2]);
                    dq[4 * c + 3] = fmaf(ds[k], kv[3], dq[4 * c + 3]);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < NE; ++k) ds[k] = 0.f;
        }
        float* dsr = DS + (h * 16 + q) * NE;
#pragma unroll
        for (int c = 0; c < 4; ++c)
            *reinterpret_cast<floatx4*>(dsr + 4 * c) = floatx4{ds[4 * c], ds[4 * c + 1], ds[4 * c + 2], ds[4 * c + 3]};
        float* dqr = dqkv + q * LDQ + h * HD;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            floatx4 v{dq[4 * c], dq[4 * c + 1], dq[4 * c + 2], dq[4 * c + 3]};
            if (ACC) v += ld4(dqr + 4 * c);
            *reinterpret_cast<floatx4*>(dqr + 4 * c) = v;
        }
    }
    wave_sync();
    {
        const int k = q;  // lane (h, key k)
        float dk[HD], dv[HD];
#pragma unroll
        for (int d = 0; d < HD; ++d) { dk[d] = 0.f; dv[d] = 0.f; }
        for (int qq = 0; qq < nq; ++qq) {
            const float dsv = DS[(h * 16 + qq) * NE + k];
            const float pv = P[(h * 16 + qq) * NE + k];
            const float* qr = qkv + qq * LDQ + h * HD;
            const float* dor = dO + qq * ldo + h * HD;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const floatx4 qv = ld4(qr + 4 * c);
                const floatx4 ov = ld4(dor + 4 * c);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    dk[4 * c + r] = fmaf(dsv, qv[r], dk[4 * c + r]);
                    dv[4 * c + r] = fmaf(pv, ov[r], dv[4 * c + r]);
                }
            }
        }
        float* kr = dqkv + k * LDQ + EMB + h * HD;
        float* vr = dqkv + k * LDQ + 2 * EMB + h * HD;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            floatx4 a{dk[4 * c], dk[4 * c + 1], dk[4 * c + 2], dk[4 * c + 3]};
            floatx4 b{dv[4 * c], dv[4 * c + 1], dv[4 * c + 2], dv[4 * c + 3]};
            if (ACC) {
                a += ld4(kr + 4 * c);
                b += ld4(vr + 4 * c);
            }
            *reinterpret_cast<floatx4*>(kr + 4 * c) = a;
            *reinterpret_cast<floatx4*>(vr + 4 * c) = b;
        }
    }
}

// ---- GRUCell on one 16-row tile, x and h in registers (D layout), PyTorch gate order r, z, n ------------
// brz = b_ih + b_hh for r, z (pre-summed). h updated in place; optional gate outputs for the backward.
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__device__ inline void gru_tile(const float* __restrict__ wih, const float* __restrict__ whh, const float* __restrict__ bih,
                                const float* __restrict__ bhh, const float* __restrict__ brz, const floatx4 (&x)[4],
                                floatx4 (&h)[4], int lane) {
    const int col = lane & 15, g = lane >> 4;
    floatx4 hn[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        floatx4 ar = ld4(brz + mt * 16 + 4 * g);
        floatx4 az = ld4(brz + EMB + mt * 16 + 4 * g);
        floatx4 ain = ld4(bih + 2 * EMB + mt * 16 + 4 * g);
        floatx4 ahn = ld4(bhh + 2 * EMB + mt * 16 + 4 * g);
        const float* wi = wih + (int64_t)(mt * 16 + col) * EMB + 4 * g;
        const float* wh = whh + (int64_t)(mt * 16 + col) * EMB + 4 * g;
        constexpr int64_t GATE = (int64_t)EMB * EMB;
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
            ar = mfma_chunk(ld4(wi + kc * 16), x[kc], ar);
            az = mfma_chunk(ld4(wi + GATE + kc * 16), x[kc], az);
            ain = mfma_chunk(ld4(wi + 2 * GATE + kc * 16), x[kc], ain);
            ar = mfma_chunk(ld4(wh + kc * 16), h[kc], ar);
            az = mfma_chunk(ld4(wh + GATE + kc * 16), h[kc], az);
            ahn = mfma_chunk(ld4(wh + 2 * GATE + kc * 16), h[kc], ahn);
#ifdef MLG_REFIL_LEAN
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float rg = sigm(ar[r]);
            const float zg = sigm(az[r]);
            const float ng = tanhf(ain[r] + rg * ahn[r]);
            hn[mt][r] = ng + zg * (h[mt][r] - ng);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) h[mt] = hn[mt];
}


// GRUCell tile with software-pipelined weight loads: the 24 weight vectors of output chunk mt + 1 are issued
// before the MFMAs of chunk mt (weights stream from L2 at one wave per SIMD; 2 x 96 VGPRs in flight).
__device__ inline void gru_tile_pipe(const float* __restrict__ wih, const float* __restrict__ whh,
                                     const float* __restrict__ bih, const float* __restrict__ bhh,
                                     const float* __restrict__ brz, const floatx4 (&x)[4], floatx4 (&h)[4], int lane) {
    const int col = lane & 15, g = lane >> 4;
    constexpr int64_t GATE = (int64_t)EMB * EMB;
    floatx4 wb[2][24];
    auto load = [&](int mt, floatx4 (&w)[24]) {
        const float* wi = wih + (int64_t)(mt * 16 + col) * EMB + 4 * g;
        const float* wh = whh + (int64_t)(mt * 16 + col) * EMB + 4 * g;
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                w[kc * 6 + q] = ld4(wi + q * GATE + kc * 16);
                w[kc * 6 + 3 + q] = ld4(wh + q * GATE + kc * 16);
            }
        }
    };
    floatx4 hn[4];
    load(0, wb[0]);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        if (mt + 1 < 4) load(mt + 1, wb[(mt + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const floatx4(&w)[24] = wb[mt & 1];
        floatx4 ar = ld4(brz + mt * 16 + 4 * g);
        floatx4 az = ld4(brz + EMB + mt * 16 + 4 * g);
        floatx4 ain = ld4(bih + 2 * EMB + mt * 16 + 4 * g);
        floatx4 ahn = ld4(bhh + 2 * EMB + mt * 16 + 4 * g);
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
            ar = mfma_chunk(w[kc * 6 + 0], x[kc], ar);
            az = mfma_chunk(w[kc * 6 + 1], x[kc], az);
            ain = mfma_chunk(w[kc * 6 + 2], x[kc], ain);
            ar = mfma_chunk(w[kc * 6 + 3], h[kc], ar);
            az = mfma_chunk(w[kc * 6 + 4], h[kc], az);
            ahn = mfma_chunk(w[kc * 6 + 5], h[kc], ahn);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float rg = sigm(ar[r]);
            const float zg = sigm(az[r]);
            const float ng = tanhf(ain[r] + rg * ahn[r]);
            hn[mt][r] = ng + zg * (h[mt][r] - ng);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) h[mt] = hn[mt];
}

// GRUCell tile with the products as split-bf16 fp32 emulation on the bf16 matrix cores: x and h
// (D layout) are split once into three bf16 pieces per 32-wide K step -- K slot (g, i) of step kk holds feature
// (2kk + i / 4) * 16 + 4g + i % 4, i.e. the lane's own registers x[2kk], x[2kk + 1] -- and the weights come
// pre-split in that K order from the packed block (section gsp, refil_pack_gsp_kernel), streamed per (mt, kk)
// with the next stage's 18 loads issued before the current stage's MFMAs. 288 bf16 MFMAs (16 cycles) instead of
// 384 f32 MFMAs (32 cycles) per tile; fp32-class results (six partial products, fp32 accumulation).
__device__ __forceinline__ int refil_gsp_reg(int mat, int mt, int gate, int kk, int piece) {
    return ((((mat * 4 + mt) * 3 + gate) * 2 + kk) * 3 + piece) * 64;
}

__device__ inline void gru_tile_b16(const float* __restrict__ P, const RAgent& L, const floatx4 (&x)[4], floatx4 (&h)[4],
                                    int lane) {
    const int g = lane >> 4;
    const u32x4* gs = reinterpret_cast<const u32x4*>(P + L.gsp) + lane;
    const float* brz = P + L.brz;
    const float* bih = P + L.bih;
    const float* bhh = P + L.bhh;
    Split3 xs[2], hs[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        xs[kk] = split3(x[2 * kk], x[2 * kk + 1]);
        hs[kk] = split3(h[2 * kk], h[2 * kk + 1]);
    }
    bf16x8 wb[2][18];  // [mat * 9 + gate * 3 + piece]
    auto load = [&](int st, bf16x8 (&w)[18]) {
        const int mt = st >> 1, kk = st & 1;
#pragma unroll
        for (int mat = 0; mat < 2; ++mat)
#pragma unroll
            for (int gate = 0; gate < 3; ++gate)
#pragma unroll
                for (int pc = 0; pc < 3; ++pc)
                    w[mat * 9 + gate * 3 + pc] = __builtin_bit_cast(bf16x8, gs[refil_gsp_reg(mat, mt, gate, kk, pc)]);
    };
    auto piece3 = [](const bf16x8 (&w)[18], int b) {
        Split3 s;
        s.p[0] = w[b];
        s.p[1] = w[b + 1];
        s.p[2] = w[b + 2];
        return s;
    };
    floatx4 hn[4];
    load(0, wb[0]);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        floatx4 ar = ld4(brz + mt * 16 + 4 * g);
        floatx4 az = ld4(brz + EMB + mt * 16 + 4 * g);
        floatx4 ain = ld4(bih + 2 * EMB + mt * 16 + 4 * g);
        floatx4 ahn = ld4(bhh + 2 * EMB + mt * 16 + 4 * g);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int st = mt * 2 + kk;
            if (st + 1 < 8) load(st + 1, wb[(st + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            const bf16x8(&w)[18] = wb[st & 1];
            ar = mfma_x6(piece3(w, 0), xs[kk], ar);
            az = mfma_x6(piece3(w, 3), xs[kk], az);
            ain = mfma_x6(piece3(w, 6), xs[kk], ain);
            ar = mfma_x6(piece3(w, 9), hs[kk], ar);
            az = mfma_x6(piece3(w, 12), hs[kk], az);
            ahn = mfma_x6(piece3(w, 15), hs[kk], ahn);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float rg = sigm(ar[r]);
            const float zg = sigm(az[r]);
            const float ng = tanhf(ain[r] + rg * ahn[r]);
            hn[mt][r] = ng + zg * (h[mt][r] - ng);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) h[mt] = hn[mt];
}

// ---- entity env variant (oracle/env_ref.c envref_reset_entity / envref_entities) ------------------------
enum { MLG_PURPOSE_TEAM = 4 };

__device__ __forceinline__ int entity_team_k(uint64_t key, uint32_t episode, int kmin, int kmax) {
    const uint64_t r = mlg_rng(key, mlg_ctr(episode, 0, MLG_PURPOSE_TEAM, 0));
    return kmin + (int)(r % (uint64_t)(kmax - kmin + 1));
}

// entity features of unit j: [1, x/P, y/P, hp/max_hp, team, role/2, melee, power/8] if alive, else zeros
__device__ __forceinline__ void entity_feat(const EnvTables& T, int x, int y, int hp, int j, float inv_p, float* o) {
    if (hp <= 0) {
#pragma unroll
        for (int f = 0; f < 8; ++f) o[f] = 0.f;
        return;
    }
    o[0] = 1.f;
    o[1] = (float)x * inv_p;
    o[2] = (float)y * inv_p;
    o[3] = (float)hp * inv_maxhp(T.role[j]);
    o[4] = (float)T.team[j];
    o[5] = (float)T.role[j] * 0.5f;
    o[6] = (float)T.melee[j];
    o[7] = (float)role_power(T.role[j]) * 0.125f;
}

}  // namespace refil

// ---- register form of the env rules for one half-wave env (lane per unit) ---------------------------------
// Units are read as packed states pk[j] = x | y << 8 | hp << 16 (four 16-byte LDS broadcast reads per env), the
// static unit tables as bit masks, loops fully unrolled: the same integer rules as env_avail_one / env_ai_action /
// env_resolve_hp (mlg_device.h, oracle/env_ref.c), without per-unit LDS lookups.
namespace refil {

struct EnvMasks {
    uint32_t team1, healer, tank, melee;
    int U, grid;
};

__device__ __forceinline__ int pk_pack(int x, int y, int hp) { return x | (y << 8) | (hp << 16); }
__device__ __forceinline__ int pkx(int p) { return p & 0xFF; }
__device__ __forceinline__ int pky(int p) { return (p >> 8) & 0xFF; }
__device__ __forceinline__ int pkh(int p) { return p >> 16; }

__device__ __forceinline__ void load16(const int* src, int (&v)[16]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int4 w = *reinterpret_cast<const int4*>(src + 4 * q);
        v[4 * q] = w.x;
        v[4 * q + 1] = w.y;
        v[4 * q + 2] = w.z;
        v[4 * q + 3] = w.w;
    }
}

// units j that unit i (alive) may target with action 5 + j
// (pi = packed state of unit i itself: never index pk[] with a runtime index, that would spill it to scratch)
__device__ __forceinline__ uint32_t target_bits(const EnvMasks& M, const int (&pk)[16], int i, int pi) {
    const int xi = pkx(pi), yi = pky(pi);
    const int r2 = ((M.melee >> i) & 1u) ? 2 : 9;
    const bool heal = (M.healer >> i) & 1u;
    const uint32_t mt = (M.team1 >> i) & 1u;
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int p = pk[j], hj = pkh(p);
        const int dx = pkx(p) - xi, dy = pky(p) - yi;
        const uint32_t tj = (M.team1 >> j) & 1u;
        const bool ok = heal ? (j != i && tj == mt && hj < (((M.tank >> j) & 1u) ? 64 : 32)) : (tj != mt);
        bits |= (uint32_t)(j < M.U && hj > 0 && dx * dx + dy * dy <= r2 && ok) << j;
    }
    return bits;
}

// avail bits of unit i: bit a = action a available (spec §3.2)
__device__ __forceinline__ uint32_t avail_bits(const EnvMasks& M, const int (&pk)[16], int i, int pi) {
    if (pkh(pi) <= 0) return 1u;
    const int x = pkx(pi), y = pky(pi);
    uint32_t m = 0;
    m |= (uint32_t)(y + 1 < M.grid) << 1;
    m |= (uint32_t)(y - 1 >= 0) << 2;
    m |= (uint32_t)(x + 1 < M.grid) << 3;
    m |= (uint32_t)(x - 1 >= 0) << 4;
    return m | (target_bits(M, pk, i, pi) << MLG_ACT_BASE);
}

__device__ __forceinline__ int move_toward_d(int dx, int dy) {
    const int adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
    if (adx >= ady && dx != 0) return dx > 0 ? 3 : 4;
    if (dy != 0) return dy > 0 ? 1 : 2;
    return 0;
}

// scripted "basic" AI of unit i (spec §3.3), pre-step state
__device__ __forceinline__ int ai_action_reg(const EnvMasks& M, const int (&pk)[16], int i, int pi) {
    if (pkh(pi) <= 0) return 0;
    const int xi = pkx(pi), yi = pky(pi);
    const uint32_t tb = target_bits(M, pk, i, pi);
    int best = -1, hb = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int hj = pkh(pk[j]);
        if (((tb >> j) & 1u) && (best < 0 || hj < hb)) { best = j; hb = hj; }
    }
    if (best >= 0) return MLG_ACT_BASE + best;
    const uint32_t mt = (M.team1 >> i) & 1u;
    if ((M.healer >> i) & 1u) {
        int near = -1, nd = 0, ndx = 0, ndy = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int p = pk[j];
            const int dx = pkx(p) - xi, dy = pky(p) - yi, d = dx * dx + dy * dy;
            const bool cand = j < M.U && j != i && pkh(p) > 0 && ((M.team1 >> j) & 1u) == mt;
            if (cand && (near < 0 || d < nd)) { near = j; nd = d; ndx = dx; ndy = dy; }
        }
        if (near >= 0) return nd > 2 ? move_toward_d(ndx, ndy) : 0;
    }
    int near = -1, nd = 0, ndx = 0, ndy = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int p = pk[j];
        const int dx = pkx(p) - xi, dy = pky(p) - yi, d = dx * dx + dy * dy;
        const bool cand = j < M.U && pkh(p) > 0 && ((M.team1 >> j) & 1u) != mt;
        if (cand && (near < 0 || d < nd)) { near = j; nd = d; ndx = dx; ndy = dy; }
    }
    return near >= 0 ? move_toward_d(ndx, ndy) : 0;
}

// new hp of unit u from all executed actions (spec §3.4)
__device__ __forceinline__ int resolve_hp_reg(const EnvMasks& M, const int (&pk)[16], const int (&act)[16], int u,
                                              int pu) {
    const int hu = pkh(pu);
    if (hu <= 0) return hu;
    int dmg = 0, heal = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const bool hit = i < M.U && pkh(pk[i]) > 0 && act[i] == MLG_ACT_BASE + u;
        const bool h = (M.healer >> i) & 1u;
        heal += (hit && h) ? 4 : 0;
        dmg += (hit && !h) ? (((M.tank >> i) & 1u) ? 3 : 6) : 0;
    }
    const int v = hu - dmg + heal, mx = ((M.tank >> u) & 1u) ? 64 : 32;
    return v < 0 ? 0 : (v > mx ? mx : v);
}

// One scan over the units j of [j0, j0 + NJ) for unit i (alive or not): target bits (as target_bits) and the scripted
// AI's min-keys -- lowest-hp target (hp << 5 | j), nearest living ally != i and nearest living enemy (d2 << 5 | j);
// "smallest value, then lowest j" is the rule of ai_action_reg's strict-< scans. The keys and bits of two scans
// over disjoint j ranges combine by min / OR, so the scan can be split across lanes (bit-identical).
template <int NJ>
__device__ __forceinline__ void unit_scan(const EnvMasks& M, const int (&pk)[16], int i, int pi, bool upper,
                                          uint32_t& tb, uint32_t& kbest, uint32_t& kally, uint32_t& kenemy) {
    const int xi = pkx(pi), yi = pky(pi);
    const int r2 = ((M.melee >> i) & 1u) ? 2 : 9;
    const bool heal = (M.healer >> i) & 1u;
    const uint32_t mt = (M.team1 >> i) & 1u;
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    tb = 0u;
    kbest = kally = kenemy = NONE;
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
        const int j = (upper ? 16 - NJ : 0) + k;
        const int p = upper ? pk[16 - NJ + k] : pk[k];  // compile-time register indices (see target_bits)
        const int hj = pkh(p);
        const int dx = pkx(p) - xi, dy = pky(p) - yi;
        const uint32_t d2 = (uint32_t)(dx * dx + dy * dy);
        const uint32_t tj = (M.team1 >> j) & 1u;
        const bool live = j < M.U && hj > 0;
        const bool ok = heal ? (j != i && tj == mt && hj < (((M.tank >> j) & 1u) ? 64 : 32)) : (tj != mt);
        const bool tg = live && d2 <= (uint32_t)r2 && ok;
        tb |= (uint32_t)tg << j;
        kbest = min(kbest, tg ? ((uint32_t)hj << 5 | (uint32_t)j) : NONE);
        kally = min(kally, (live && j != i && tj == mt) ? (d2 << 5 | (uint32_t)j) : NONE);
        kenemy = min(kenemy, (live && tj != mt) ? (d2 << 5 | (uint32_t)j) : NONE);
    }
}

// The scripted AI action (ai_action_reg) from unit_scan's combined results; pkj(j) = packed state of unit j.
template <typename PK>
__device__ __forceinline__ int ai_from_scan(const EnvMasks& M, int i, int pi, uint32_t kbest, uint32_t kally,
                                            uint32_t kenemy, PK pkj) {
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    if (pkh(pi) <= 0) return 0;
    if (kbest != NONE) return MLG_ACT_BASE + (int)(kbest & 31u);
    uint32_t k = kenemy;
    if ((M.healer >> i) & 1u) {
        if (kally != NONE) {
            if ((kally >> 5) <= 2u) return 0;
            k = kally;
        }
    }
    if (k == NONE) return 0;
    const int p = pkj((int)(k & 31u));
    return move_toward_d(pkx(p) - pkx(pi), pky(p) - pky(pi));
}

// obs-mask row of unit u: bit j = u dead, j dead or out of sight
__device__ __forceinline__ uint32_t om_bits(const EnvMasks& M, const int (&pk)[16], int u, int pu) {
    (void)u;
    if (pkh(pu) <= 0) return (1u << M.U) - 1u;
    const int xu = pkx(pu), yu = pky(pu);
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int p = pk[j];
        const int dx = pkx(p) - xu, dy = pky(p) - yu;
        bits |= (uint32_t)(j < M.U && (pkh(p) <= 0 || dx * dx + dy * dy > MLG_SIGHT2)) << j;
    }
    return bits;
}

}  // namespace refil
