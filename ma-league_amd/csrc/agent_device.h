// agent_device.h -- the DRQN agent cell (fc1 -> ReLU -> GRUCell -> fc2) on one 16-row tile per wave,
// f32 MFMA (16x16x4), register resident.  Restates DRQNAgentNetwork.forward
// (src/marl/modules/agents/drqn_agent.py:29-35) with BasicMAC._build_inputs folded in
// (src/marl/controllers/basic_controller.py:80-92): the one-hot last action and the agent id
// columns of fc1 are added as weight-column gathers instead of dense K (identical sum, no zeros).
//
// Packed weight block (floats; every offset 16-byte aligned; H % 16 == 0):
//   w1d [H][Dip]  fc1.weight dense (Dip = d_in rounded up to 16, zero padded) for arbitrary inputs
//   w1o [H][Dob]  fc1.weight obs columns (Dob = d_obs rounded up to 16, zero padded)
//   w1a [A][H]    fc1.weight last-action columns, transposed   (present iff obs_last_action)
//   w1n [N][H]    fc1.weight agent-id columns, transposed       (present iff obs_agent_id)
//   b1  [H]
//   wih [3H][H], bih [3H], whh [3H][H], bhh [3H]   (PyTorch GRUCell gate order r, z, n)
//   brz [2H]      b_ih + b_hh for the r,z gates (pre-summed)
//   w2  [Ap][H]   fc2.weight zero padded to Ap = A rounded up to 16 rows
//   b2  [Ap]
//   gsp [8 waves][18 regs][64 lanes][4]  (H = 64 only) the GRU weights as split-bf16 pieces in the register
//                 layout of the self-play kernel's waves (GruG8: per K step kk, {W_ir;W_iz}, {W_hr;W_hz},
//                 {W_in;W_hn} rows, pieces 0..2; a u32 = two bf16), so a weight swap is 18 straight loads
//   w1s [H/16 chunks][KK][3 pieces][64 lanes][4]  (H = 64 only) fc1 obs columns as split-bf16 A operands
//                 (K steps of 32, zero padded past d_obs)
//   w2s [Ap/16][2 K steps][3 pieces][64 lanes][4]  (H = 64 only) fc2 as split-bf16 A operands (rows >= A zero; the
//                 one-round self-play kernel sp8 runs fc2 on the bf16 planes of h')
#pragma once
#include "mlg_device.h"

struct AgentLayout {
    int H, A, Ap, N, d_obs, Dob, d_in, Dip, last_action, agent_id;
    int32_t w1d, w1o, w1a, w1n, b1, wih, bih, whh, bhh, brz, w2, b2, gsp, w1s, w2s, total;  // 32-bit: fewer SGPRs
};

__host__ __device__ constexpr int64_t mlg_align4(int64_t v) { return (v + 3) & ~int64_t(3); }

__host__ __device__ constexpr AgentLayout make_agent_layout(const MlgAgentDims& d) {
    AgentLayout L{};
    L.H = d.hidden;
    L.A = d.n_actions;
    L.Ap = (d.n_actions + 15) / 16 * 16;
    L.N = d.n_agents;
    L.d_obs = d.d_obs;
    L.Dob = (d.d_obs + 15) / 16 * 16;
    L.d_in = d.d_in;
    L.Dip = (d.d_in + 15) / 16 * 16;
    L.last_action = d.obs_last_action;
    L.agent_id = d.obs_agent_id;
    int64_t o = 0;
    L.w1d = o; o += (int64_t)L.H * L.Dip;
    L.w1o = o; o += (int64_t)L.H * L.Dob;
    L.w1a = o; o += L.last_action ? (int64_t)L.A * L.H : 0;
    L.w1n = o; o += L.agent_id ? (int64_t)L.N * L.H : 0;
    L.b1 = o; o += L.H;
    L.wih = o; o += (int64_t)3 * L.H * L.H;
    L.bih = o; o += 3 * L.H;
    L.whh = o; o += (int64_t)3 * L.H * L.H;
    L.bhh = o; o += 3 * L.H;
    L.brz = o; o += 2 * L.H;
    L.w2 = o; o += (int64_t)L.Ap * L.H;
    L.b2 = o; o += L.Ap;
    o = mlg_align4(o);
    L.gsp = o; o += L.H == 64 ? 8 * 18 * 64 * 4 : 0;
    L.w1s = o; o += L.H == 64 ? (int64_t)(L.H / 16) * ((L.Dob + 31) / 32) * 3 * 64 * 4 : 0;
    L.w2s = o; o += L.H == 64 ? (int64_t)(L.Ap / 16) * 2 * 3 * 64 * 4 : 0;
    L.total = mlg_align4(o);
    return L;
}

// Packed float i of the kernel weight layout from the canonical nn.Module tensors (pack_agent_kernel and the
// learner's fused prologue).
__device__ __forceinline__ float pack_agent_elem(const AgentLayout& L, const MlgAgentParams& p, int64_t i) {
    const int H = L.H;
    float v = 0.f;
    if (i < L.w1o) {  // dense fc1 [H][Dip]
        const int64_t r = i / L.Dip, c = i % L.Dip;
        v = c < L.d_in ? p.fc1_w[r * L.d_in + c] : 0.f;
    } else if (i < L.w1a) {  // obs columns [H][Dob]
        const int64_t k = i - L.w1o, r = k / L.Dob, c = k % L.Dob;
        v = c < L.d_obs ? p.fc1_w[r * L.d_in + c] : 0.f;
    } else if (i < L.w1n) {  // last-action columns transposed [A][H]
        const int64_t k = i - L.w1a, a = k / H, r = k % H;
        v = p.fc1_w[r * L.d_in + L.d_obs + a];
    } else if (i < L.b1) {  // agent-id columns transposed [N][H]
        const int64_t k = i - L.w1n, n = k / H, r = k % H;
        v = p.fc1_w[r * L.d_in + L.d_obs + (L.last_action ? L.A : 0) + n];
    } else if (i < L.wih) {
        v = p.fc1_b[i - L.b1];
    } else if (i < L.bih) {
        v = p.w_ih[i - L.wih];
    } else if (i < L.whh) {
        v = p.b_ih[i - L.bih];
    } else if (i < L.bhh) {
        v = p.w_hh[i - L.whh];
    } else if (i < L.brz) {
        v = p.b_hh[i - L.bhh];
    } else if (i < L.w2) {
        const int64_t k = i - L.brz;
        v = p.b_ih[k] + p.b_hh[k];
    } else if (i < L.b2) {
        const int64_t k = i - L.w2, r = k / H, c = k % H;
        v = r < L.A ? p.fc2_w[r * H + c] : 0.f;
    } else if (i < L.gsp) {
        const int64_t k = i - L.b2;
        v = k < L.Ap && k < L.A ? p.fc2_b[k] : 0.f;
    } else if (i < L.w1s) {  // split GRU pieces (H = 64): k = ((w * 18 + kk * 9 + mat * 3 + piece) * 64 + lane) * 4 + q
        const int64_t k = i - L.gsp;
        const int q = (int)(k & 3), lane = (int)((k >> 2) & 63), r = (int)((k >> 8) % 18), w = (int)((k >> 8) / 18);
        const int kk = r / 9, mat = (r / 3) % 3, piece = r % 3;
        const int row = lane & 15, g = lane >> 4, f = 8 * w + (row & 7), hi = row >> 3;
        const float* src = mat == 0 ? p.w_ih + (int64_t)(hi * H + f) * H
                                    : (mat == 1 ? p.w_hh + (int64_t)(hi * H + f) * H
                                                : (hi ? p.w_hh : p.w_ih) + (int64_t)(2 * H + f) * H);
        const int kb = 32 * kk + 8 * g + 2 * q;
        v = split_bf16_pair(src[kb], src[kb + 1], piece);
    } else if (i < L.w2s) {  // split fc1 obs columns: k = (((j * KK + kk) * 3 + piece) * 64 + lane) * 4 + q
        const int64_t k = i - L.w1s;
        const int KK = (L.Dob + 31) / 32;
        const int q = (int)(k & 3), lane = (int)((k >> 2) & 63), r = (int)(k >> 8);
        const int piece = r % 3, kk = (r / 3) % KK, j = r / (3 * KK);
        const int64_t row = j * 16 + (lane & 15);
        const int kb = 32 * kk + 8 * (lane >> 4) + 2 * q;
        const float a = kb < L.d_obs ? p.fc1_w[row * L.d_in + kb] : 0.f;
        const float b = kb + 1 < L.d_obs ? p.fc1_w[row * L.d_in + kb + 1] : 0.f;
        v = split_bf16_pair(a, b, piece);
    } else if (i < L.total) {  // split fc2: k = ((((at * 2 + kk) * 3 + piece) * 64 + lane) * 4 + q
        const int64_t k = i - L.w2s;
        const int q = (int)(k & 3), lane = (int)((k >> 2) & 63), r = (int)(k >> 8);
        const int piece = r % 3, kk = (r / 3) % 2, at = r / 6;
        const int row = 16 * at + (lane & 15), kb = 32 * kk + 8 * (lane >> 4) + 2 * q;
        const float a = row < L.A ? p.fc2_w[(int64_t)row * H + kb] : 0.f;
        const float b = row < L.A ? p.fc2_w[(int64_t)row * H + kb + 1] : 0.f;
        v = split_bf16_pair(a, b, piece);
    }
    return v;
}

// Per-lane inputs of a 16-row tile: this lane's row (col = lane & 15) data.
//   DENSE:      x = full input row [d_in] (DRQNAgentNetwork.forward on arbitrary inputs)
//   structured: x = obs row [d_obs]; last action from `onehot` (A floats, added as v * column) or,
//               when onehot == nullptr, from `prev_action` (-1: zeros, t == 0); agent id column `agent`.
struct RowIn {
    const float* x;
    const float* onehot;
    int prev_action;
    int agent;
};

__device__ __forceinline__ floatx4 load_chunk(const float* x, int k0, int n) {
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (x) {
        if (k0 + 3 < n) {
            v = floatx4{x[k0], x[k0 + 1], x[k0 + 2], x[k0 + 3]};
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (k0 + r < n) ? x[k0 + r] : 0.f;
        }
    }
    return v;
}

// Where the cell reads its weights from: the packed block in HBM/L2 (row strides = the packed widths) or a
// padded copy in LDS (row strides + 4 floats, so the 16 rows of an A-operand read hit 16 distinct
// 16-byte bank slots).  Offsets are in floats from p.
struct WView {
    const float* p;
    int32_t w1d, w1o, w1a, w1n, b1, wih, bih, whh, bhh, brz, w2, b2;
    int ldd, ldo, ldh;
};

__host__ __device__ inline WView global_view(const float* P, const AgentLayout& L) {
    WView v;
    v.p = P;
    v.w1d = L.w1d; v.w1o = L.w1o; v.w1a = L.w1a; v.w1n = L.w1n; v.b1 = L.b1; v.wih = L.wih; v.bih = L.bih;
    v.whh = L.whh; v.bhh = L.bhh; v.brz = L.brz; v.w2 = L.w2; v.b2 = L.b2;
    v.ldd = L.Dip; v.ldo = L.Dob; v.ldh = L.H;
    return v;
}

// LDS image used by the rollout kernel (no dense w1d): offsets relative to the LDS base.
struct LdsWeights {
    int32_t w1o, w1a, w1n, b1, wih, bih, whh, bhh, brz, w2, b2, total;
    int ldo, ldh;
};
__host__ __device__ inline LdsWeights make_lds_weights(const AgentLayout& L) {
    LdsWeights w;
    w.ldo = L.Dob + 4;
    w.ldh = L.H + 4;
    int64_t o = 0;
    w.w1o = o; o += (int64_t)L.H * w.ldo;
    w.w1a = o; o += L.last_action ? (int64_t)L.A * w.ldh : 0;
    w.w1n = o; o += L.agent_id ? (int64_t)L.N * w.ldh : 0;
    w.b1 = o; o += L.H;
    w.wih = o; o += (int64_t)3 * L.H * w.ldh;
    w.bih = o; o += 3 * L.H;
    w.whh = o; o += (int64_t)3 * L.H * w.ldh;
    w.bhh = o; o += 3 * L.H;
    w.brz = o; o += 2 * L.H;
    w.w2 = o; o += (int64_t)L.Ap * w.ldh;
    w.b2 = o; o += L.Ap;
    w.total = mlg_align4(o);
    return w;
}

__device__ inline WView lds_view(const float* base, const LdsWeights& w, const AgentLayout& L) {
    WView v;
    v.p = base;
    v.w1d = 0; v.w1o = w.w1o; v.w1a = w.w1a; v.w1n = w.w1n; v.b1 = w.b1; v.wih = w.wih; v.bih = w.bih;
    v.whh = w.whh; v.bhh = w.bhh; v.brz = w.brz; v.w2 = w.w2; v.b2 = w.b2;
    v.ldd = 0; v.ldo = w.ldo; v.ldh = w.ldh;
    return v;
}

// Cooperative copy packed (global) -> padded LDS image (whole workgroup; caller syncs).
__device__ inline void load_weights_to_lds(const float* __restrict__ P, const AgentLayout& L, const LdsWeights& w,
                                           float* lds) {
    const int H = L.H;
    auto rows = [&](int64_t src, int64_t dst, int nrows, int ncols, int ld) {
        for (int i = threadIdx.x; i < nrows * ncols; i += blockDim.x) {
            const int r = i / ncols, c = i % ncols;
            lds[dst + (int64_t)r * ld + c] = P[src + (int64_t)r * ncols + c];
        }
    };
    rows(L.w1o, w.w1o, H, L.Dob, w.ldo);
    if (L.last_action) rows(L.w1a, w.w1a, L.A, H, w.ldh);
    if (L.agent_id) rows(L.w1n, w.w1n, L.N, H, w.ldh);
    rows(L.b1, w.b1, 1, H, H);
    rows(L.wih, w.wih, 3 * H, H, w.ldh);
    rows(L.bih, w.bih, 1, 3 * H, 3 * H);
    rows(L.whh, w.whh, 3 * H, H, w.ldh);
    rows(L.bhh, w.bhh, 1, 3 * H, 3 * H);
    rows(L.brz, w.brz, 1, 2 * H, 2 * H);
    rows(L.w2, w.w2, L.Ap, H, w.ldh);
    rows(L.b2, w.b2, 1, L.Ap, L.Ap);
}

// fc1 (pre-activation, bias included) for one tile -> x (HC chunks, D layout).
template <int H, bool DENSE>
__device__ __forceinline__ void agent_fc1(const WView& W, const AgentLayout& L, const RowIn& in, floatx4 (&x)[H / 16],
                                          int lane) {
    constexpr int HC = H / 16;
    const int col = lane & 15, g = lane >> 4;
    const float* P = W.p;
#pragma unroll
    for (int mt = 0; mt < HC; ++mt) {
        floatx4 b = ld4(P + W.b1 + mt * 16 + 4 * g);
        if (!DENSE) {
            if (L.last_action) {
                if (in.onehot) {
                    for (int a = 0; a < L.A; ++a) {
                        const float v = in.onehot[a];
                        if (v != 0.f) b += v * ld4(P + W.w1a + (int64_t)a * W.ldh + mt * 16 + 4 * g);
                    }
                } else if (in.prev_action >= 0) {
                    b += ld4(P + W.w1a + (int64_t)in.prev_action * W.ldh + mt * 16 + 4 * g);
                }
            }
            if (L.agent_id) b += ld4(P + W.w1n + (int64_t)in.agent * W.ldh + mt * 16 + 4 * g);
        }
        x[mt] = b;
    }
    const int K = DENSE ? L.d_in : L.d_obs;
    const int KP = DENSE ? L.Dip : L.Dob;
    const int ld = DENSE ? W.ldd : W.ldo;
    const float* base = P + (DENSE ? W.w1d : W.w1o) + (int64_t)col * ld + 4 * g;
    for (int kc = 0; kc < KP / 16; ++kc) {
        const int k0 = kc * 16 + 4 * g;
        const floatx4 xin = load_chunk(in.x, k0, K);
#pragma unroll
        for (int mt = 0; mt < HC; ++mt) x[mt] = mfma_chunk(ld4(base + (int64_t)mt * 16 * ld + kc * 16), xin, x[mt]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// fc1 + ReLU + GRUCell for one tile; h (HC chunks, D layout) updated in place.
template <int H, bool DENSE = false>
__device__ __forceinline__ void agent_cell_hidden(const WView& W, const AgentLayout& L, const RowIn& in,
                                                  floatx4 (&h)[H / 16], int lane) {
    constexpr int HC = H / 16;
    const int col = lane & 15, g = lane >> 4;
    const float* P = W.p;
    floatx4 x[HC];
    agent_fc1<H, DENSE>(W, L, in, x, lane);
#pragma unroll
    for (int mt = 0; mt < HC; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) x[mt][r] = fmaxf(x[mt][r], 0.f);
    // ---- GRUCell, one 16-feature output chunk at a time (4 live accumulators):
    //   r = sig(W_ir x + W_hr h + b_ir + b_hr), z likewise, n = tanh(W_in x + b_in + r (W_hn h + b_hn)),
    //   h' = (h - n) z + n   (PyTorch GRUCell gate order and formula)
    floatx4 hn[HC];
    const int64_t gate = (int64_t)H * W.ldh;  // row offset between the r, z and n blocks
#pragma unroll
    for (int mt = 0; mt < HC; ++mt) {
        floatx4 ar = ld4(P + W.brz + mt * 16 + 4 * g);
        floatx4 az = ld4(P + W.brz + H + mt * 16 + 4 * g);
        floatx4 ain = ld4(P + W.bih + 2 * H + mt * 16 + 4 * g);
        floatx4 ahn = ld4(P + W.bhh + 2 * H + mt * 16 + 4 * g);
        const float* wr_i = P + W.wih + (int64_t)(mt * 16 + col) * W.ldh + 4 * g;
        const float* wr_h = P + W.whh + (int64_t)(mt * 16 + col) * W.ldh + 4 * g;
#pragma unroll
        for (int kc = 0; kc < HC; ++kc) {
            const int k0 = kc * 16;
            ar = mfma_chunk(ld4(wr_i + k0), x[kc], ar);
            az = mfma_chunk(ld4(wr_i + gate + k0), x[kc], az);
            ain = mfma_chunk(ld4(wr_i + 2 * gate + k0), x[kc], ain);
            ar = mfma_chunk(ld4(wr_h + k0), h[kc], ar);
            az = mfma_chunk(ld4(wr_h + gate + k0), h[kc], az);
            ahn = mfma_chunk(ld4(wr_h + 2 * gate + k0), h[kc], ahn);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float rg = 1.f / (1.f + expf(-ar[r]));
            const float zg = 1.f / (1.f + expf(-az[r]));
            const float ng = tanhf(ain[r] + rg * ahn[r]);
            hn[mt][r] = ng + zg * (h[mt][r] - ng);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the next chunk's weight loads from being hoisted (VGPR budget)
    }
#pragma unroll
    for (int mt = 0; mt < HC; ++mt) h[mt] = hn[mt];
}

// fc2 for action tile at (16 actions starting at 16*at): q (D layout) for this lane's row.
template <int H>
__device__ __forceinline__ floatx4 agent_q_tile(const WView& W, const floatx4 (&h)[H / 16], int at, int lane) {
    constexpr int HC = H / 16;
    const int col = lane & 15, g = lane >> 4;
    floatx4 q = ld4(W.p + W.b2 + at * 16 + 4 * g);
#pragma unroll
    for (int kc = 0; kc < HC; ++kc)
        q = mfma_chunk(ld4(W.p + W.w2 + (int64_t)(at * 16 + col) * W.ldh + kc * 16 + 4 * g), h[kc], q);
    return q;
}

// Masked greedy argmax + epsilon-greedy pick for the lane's row (EpsilonGreedyActionSelector.select,
// action_selectors.py:44-62). q tile values for actions 16*at + 4*g + r. Returns, in every lane of the
// row group, the chosen action.  avail: this row's A ints (nullptr -> all available).
struct ArgmaxState {
    float bv;
    int bi;
};

__device__ __forceinline__ void argmax_accumulate(ArgmaxState& s, const floatx4 q, const int32_t* avail, int at, int A, int lane) {
    const int g = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int a = at * 16 + 4 * g + r;
        if (a >= A) continue;
        const float v = (avail && avail[a] == 0) ? -INFINITY : q[r];
        if (amax_better(v, a, s.bv, s.bi)) { s.bv = v; s.bi = a; }
    }
}

// Reduction over the four 16-lane rows (lane l with l ^ 16, then l ^ 32) by v_permlane16/32_swap (VALU) instead of
// LDS permutes: the same exchanged values, ~10x less latency on the action-selection path. All 64 lanes must be
// active (callers: wave-uniform tile loops).
__device__ __forceinline__ int argmax_reduce(ArgmaxState s) {
    const bool odd16 = (threadIdx.x & 16) != 0, hi32 = (threadIdx.x & 32) != 0;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const unsigned uv = __float_as_uint(s.bv), ui = (unsigned)s.bi;
        float ov;
        int oi;
        if (r == 0) {  // lane ^ 16: even rows read the second result, odd rows the first
            const auto xv = __builtin_amdgcn_permlane16_swap(uv, uv, false, false);
            const auto xi = __builtin_amdgcn_permlane16_swap(ui, ui, false, false);
            ov = __uint_as_float(odd16 ? xv[0] : xv[1]);
            oi = (int)(odd16 ? xi[0] : xi[1]);
        } else {       // lane ^ 32
            const auto xv = __builtin_amdgcn_permlane32_swap(uv, uv, false, false);
            const auto xi = __builtin_amdgcn_permlane32_swap(ui, ui, false, false);
            ov = __uint_as_float(hi32 ? xv[0] : xv[1]);
            oi = (int)(hi32 ? xi[0] : xi[1]);
        }
        const bool take = amax_better(ov, oi, s.bv, s.bi);
        s.bv = take ? ov : s.bv;
        s.bi = take ? oi : s.bi;
    }
    return s.bi;
}

// Random available action: k-th available with k = floor(u * n_avail), integer form (spec §3.7).
__device__ __forceinline__ int random_available(const int32_t* avail, int A, uint64_t r) {
    int n = 0;
    for (int a = 0; a < A; ++a) n += (avail == nullptr || avail[a] != 0);
    if (n == 0) return 0;
    const int k = (int)(((r >> 40) * (uint64_t)n) >> 24);
    int c = 0;
    for (int a = 0; a < A; ++a) {
        if (avail == nullptr || avail[a] != 0) {
            if (c == k) return a;
            ++c;
        }
    }
    return 0;
}
