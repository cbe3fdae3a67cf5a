// refil.hip -- REFIL (config 5) on gfx950: the entity-scheme rollout and the EntityAttentionRNNAgent forward.
//
//   mlg_refil_pack_agent    canonical flat parameters -> kernel layout (refil_device.h RAgent)
//   mlg_refil_rollout       ParallelStepper.run over the entity env variant with EntityMAC acting
//                           (src/steppers/parallel_stepper.py:106-216 semantics, EntityMAC._build_inputs
//                           src/marl/controllers/entity_controller.py:11-30 with t -> slice(t, t + 1),
//                           EntityAttentionRNNAgent.forward src/marl/modules/agents/entity_rnn_agent.py:32-65,
//                           EpsilonGreedyActionSelector.select src/marl/components/action_selectors.py:44-62)
//   mlg_refil_agent_forward one EntityAttentionRNNAgent.forward step (ts = 1) over R items
//
// Rollout structure: one wave per workgroup owns two envs for the whole episode. Env lanes 0..31 (lane per unit,
// half-wave per env) step the env with the unit state in LDS; the agent phase runs per env: entity inputs ->
// fc1 (MFMA, 16 entity rows) -> in_trans -> attention (lane per head x query), then both envs' 2 x 8 agent rows
// form one 16-row tile for out_trans -> fc2 -> GRUCell -> fc3 with the hidden state in VGPRs.
#include <cstdlib>
#include <cstring>

#include "mlg_host.h"
#include "refil_device.h"

using namespace refil;

// Phase functions of the rollout are kept out of line by default: inlined, the compiler hoists weight loads across
// phases and the kernel needs > 512 registers (1 wave per SIMD, spills); out of line it fits 2 waves per SIMD.
#ifdef MLG_REFIL_NOINLINE
#define RO_PHASE __device__ __attribute__((noinline))
#else
#define RO_PHASE __device__ inline
#endif

#ifdef MLG_STAMPS
// Diagnostic build only: per-wave cycle counts of the REFIL rollout phases, g_refil_stamps[wave][32]
// (slots 0..29 phases, 30 total, 31 = 1).
__device__ unsigned long long* g_refil_stamps = nullptr;
struct RStamps {
    unsigned long long acc[30], last, begin;
    __device__ void init() {
        for (int k = 0; k < 30; ++k) acc[k] = 0;
        last = begin = __builtin_amdgcn_s_memtime();
    }
    __device__ void mark(int k) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        acc[k] += now - last;
        last = now;
    }
    // steps by kind: k = 0 both pairs running, 1 one pair; cycles in slot 9 + k, step counts in slot 11 + k
    unsigned long long s0;
    __device__ void step_begin() { s0 = __builtin_amdgcn_s_memtime(); }
    __device__ void step_end(int k) {
        acc[9 + k] += __builtin_amdgcn_s_memtime() - s0;
        acc[11 + k] += 1;
    }
    __device__ void flush() {
        if ((threadIdx.x & 63) || !g_refil_stamps) return;
        unsigned long long* o = g_refil_stamps + ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 32;
        for (int k = 0; k < 30; ++k) o[k] = acc[k];
        o[30] = __builtin_amdgcn_s_memtime() - begin;
        o[31] = 1;
    }
};
#else
struct RStamps {
    __device__ void init() {}
    __device__ void mark(int) {}
    __device__ void step_begin() {}
    __device__ void step_end(int) {}
    __device__ void flush() {}
};
#endif

namespace {

// ---- packing -----------------------------------------------------------------------------------------
struct CopyJob {
    int64_t src, src2, dst;
    int rows_dst, cols_dst, rows_src, cols_src;
};
struct CopyJobs {
    CopyJob j[16];
    int n;
    int64_t total;  // floats of the packed block (everything not covered by a job is zeroed)
};

__global__ void copy_jobs_kernel(CopyJobs J, const float* __restrict__ src, float* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= J.total) return;
    float v = 0.f;
    for (int q = 0; q < J.n; ++q) {
        const CopyJob& c = J.j[q];
        const int64_t n = (int64_t)c.rows_dst * c.cols_dst;
        if (i >= c.dst && i < c.dst + n) {
            const int64_t l = i - c.dst;
            const int r = (int)(l / c.cols_dst), col = (int)(l % c.cols_dst);
            if (r < c.rows_src && col < c.cols_src) {
                v = src[c.src + (int64_t)r * c.cols_src + col];
                if (c.src2 >= 0) v += src[c.src2 + (int64_t)r * c.cols_src + col];
            }
            break;
        }
    }
    dst[i] = v;
}

// gsp section of the packed agent (refil_device.h gru_tile_b16): element ((reg * 64 + lane) * 4 + q) = bf16 pair
// (2q, 2q + 1) of piece `pc` of the A operand of (mat, mt, gate, kk): row gate * 64 + mt * 16 + (lane & 15), K slots
// 2q, 2q + 1 of lane group g = lane >> 4, feature (2kk + i / 4) * 16 + 4g + i % 4 for slot i.
// wsp section (in_trans, out_trans, fc2, fc1, fc3 of the rollout): the same element order per (tile, kk, piece),
// row (lane & 15) of the tile's 16 output features; fc1's K slots >= D0 and fc3's rows >= A are zero. One launch
// writes both sections.
__global__ void refil_pack_gsp_kernel(RAgent L, const float* __restrict__ flat, float* __restrict__ packed) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= REFIL_GSP + REFIL_WSP) return;
    if (k >= REFIL_GSP) {
        k -= REFIL_GSP;
        const int q = (int)(k & 3), lane = (int)((k >> 2) & 63), reg = (int)(k >> 8);
        const int pc = reg % 3, kk = (reg / 3) % 2, mt = reg / 6;
        const int i0 = 2 * q, f0 = (2 * kk + i0 / 4) * 16 + 4 * (lane >> 4) + i0 % 4;
        int64_t src;
        int row = lane & 15, rows = EMB, cols = EMB;
        if (mt < REFIL_WSP_WOUT) {
            src = L.c_win + (int64_t)mt * 16 * EMB;
        } else if (mt < REFIL_WSP_W2) {
            src = L.c_wout + (int64_t)(mt - REFIL_WSP_WOUT) * 16 * EMB;
        } else if (mt < REFIL_WSP_W1) {
            src = L.c_w2 + (int64_t)(mt - REFIL_WSP_W2) * 16 * EMB;
        } else if (mt < REFIL_WSP_W3) {
            src = L.c_w1 + (int64_t)(mt - REFIL_WSP_W1) * 16 * L.D0;
            cols = L.D0;
        } else {
            row += (mt - REFIL_WSP_W3) * 16;
            src = L.c_w3;
            rows = L.A;
        }
        const float* W = flat + src + (int64_t)row * cols;
        const bool rv = row < rows;
        const float w0 = rv && f0 < cols ? W[f0] : 0.f, w1 = rv && f0 + 1 < cols ? W[f0 + 1] : 0.f;
        packed[L.wsp + k] = split_bf16_pair(w0, w1, pc);
        return;
    }
    const int q = (int)(k & 3), lane = (int)((k >> 2) & 63), reg = (int)(k >> 8);
    const int pc = reg % 3, kk = (reg / 3) % 2, gate = (reg / 6) % 3, mt = (reg / 18) % 4, mat = reg / 72;
    const int row = gate * EMB + mt * 16 + (lane & 15), g = lane >> 4;
    const int i0 = 2 * q, f0 = (2 * kk + i0 / 4) * 16 + 4 * g + i0 % 4;
    const float* W = flat + (mat ? L.c_whh : L.c_wih) + (int64_t)row * EMB;
    packed[L.gsp + k] = split_bf16_pair(W[f0], W[f0 + 1], pc);
}

CopyJob cj(int64_t src, int64_t dst, int rd, int cd, int rs, int cs, int64_t src2 = -1) {
    return CopyJob{src, src2, dst, rd, cd, rs, cs};
}

CopyJobs agent_pack_jobs(const RAgent& L) {
    CopyJobs J;
    J.n = 0;
    J.j[J.n++] = cj(L.c_w1, L.w1, EMB, L.K1, EMB, L.D0);
    J.j[J.n++] = cj(L.c_b1, L.b1, 1, EMB, 1, EMB);
    J.j[J.n++] = cj(L.c_win, L.win, 3 * EMB, EMB, 3 * EMB, EMB);
    J.j[J.n++] = cj(L.c_wout, L.wout, EMB, EMB, EMB, EMB);
    J.j[J.n++] = cj(L.c_bout, L.bout, 1, EMB, 1, EMB);
    J.j[J.n++] = cj(L.c_w2, L.w2, EMB, EMB, EMB, EMB);
    J.j[J.n++] = cj(L.c_b2, L.b2, 1, EMB, 1, EMB);
    J.j[J.n++] = cj(L.c_wih, L.wih, 3 * EMB, EMB, 3 * EMB, EMB);
    J.j[J.n++] = cj(L.c_whh, L.whh, 3 * EMB, EMB, 3 * EMB, EMB);
    J.j[J.n++] = cj(L.c_bih, L.bih, 1, 3 * EMB, 1, 3 * EMB);
    J.j[J.n++] = cj(L.c_bhh, L.bhh, 1, 3 * EMB, 1, 3 * EMB);
    J.j[J.n++] = cj(L.c_bih, L.brz, 1, 2 * EMB, 1, 2 * EMB, L.c_bhh);
    J.j[J.n++] = cj(L.c_w3, L.w3, L.Ap, EMB, L.A, EMB);
    J.j[J.n++] = cj(L.c_b3, L.b3, 1, L.Ap, 1, L.A);
    J.total = L.total;
    return J;
}

int launch_copy(const CopyJobs& J, const float* src, float* dst, hipStream_t s) {
    hipLaunchKernelGGL(copy_jobs_kernel, dim3((unsigned)((J.total + 255) / 256)), dim3(256), 0, s, J, src, dst);
    return mlg::check_launch("refil pack");
}

int check_dims(const MlgRefilDims* d) {
    MLG_REQUIRE(d != nullptr, "null refil dims");
    MLG_REQUIRE(d->n_agents >= 1 && d->n_agents <= NAS, "refil: n_agents=%d unsupported (1..8)", d->n_agents);
    MLG_REQUIRE(d->n_entities >= d->n_agents && d->n_entities <= NE, "refil: n_entities=%d unsupported (n_agents..16)",
                d->n_entities);
    MLG_REQUIRE(d->attn_embed_dim == EMB && d->rnn_hidden_dim == EMB && d->attn_n_heads == NH,
                "refil: attn_embed_dim=%d rnn_hidden_dim=%d attn_n_heads=%d unsupported (64, 64, 4)", d->attn_embed_dim,
                d->rnn_hidden_dim, d->attn_n_heads);
    const int D0 = d->entity_shape + (d->entity_last_action ? d->n_actions : 0);
    MLG_REQUIRE(d->entity_shape >= 1 && D0 <= KMAX, "refil: entity input width %d unsupported (<= %d)", D0, KMAX);
    MLG_REQUIRE(d->n_actions >= 1 && d->n_actions <= 32, "refil: n_actions=%d unsupported (<= 32)", d->n_actions);
    return 0;
}

__host__ inline RAgent agent_layout(const MlgRefilDims* d) {
    return make_ragent(d->entity_shape + (d->entity_last_action ? d->n_actions : 0), d->n_actions);
}

// ---- the agent tile (two items x 8 agent rows) ----------------------------------------------------------
// Entity block of one item: ein (LDS [16][LDI]) -> x1 = relu(fc1) -> qkv = in_trans(x1) -> attention with the
// item's pre-mask rows -> o rows [obase, obase + nq). The caller syncs before reusing ein/x1/qkv.
__device__ inline void entity_block(const float* __restrict__ P, const RAgent& L, const float* ein, float* x1, float* qkv,
                                    const uint32_t* mrow, int nq, int ne, float* o, int lane) {
    dense_lds<true>(P + L.w1, L.K1, P + L.b1, EMB / 16, ein, LDI, L.K1 / 16, x1, LDX, lane);
    wave_sync();
    dense_lds<false>(P + L.win, EMB, nullptr, 3 * EMB / 16, x1, LDX, EMB / 16, qkv, LDQ, lane);
    wave_sync();
    attn_fwd(qkv, mrow, nq, ne, o, LDX, nullptr, lane);
    wave_sync();
}

// Rollout form: the entity inputs arrive as the fc1 B operand in registers (xin, lane = entity row), fc1's output
// stays in registers as in_trans' B operand; only q (agent rows, [NAS][LDX]) and k | v ([NE][LDKV]) go to LDS.
constexpr int LDKV = 2 * EMB + 4;
template <int KC1>
__device__ inline void entity_block_reg(const float* __restrict__ P, const RAgent& L, const float* win, int ldin,
                                        const floatx4 (&xin)[KC1], float* qs, float* kvs, const uint32_t* mrow, int nq,
                                        int ne, float* o, int lane) {
    const int col = lane & 15;
    floatx4 x1[4];
    bias_init<4>(x1, P + L.b1, 0, lane);
#if !defined(MLG_REFIL_INTRANS_F32)
    if constexpr (KC1 == 2) {  // K1 = 32: one split-bf16 K step over xin[0], xin[1] (wsp tiles 20-23, kk = 0)
        const u32x4* ws = reinterpret_cast<const u32x4*>(P + L.wsp) + lane;
        bf16x8 w[12];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int pc = 0; pc < 3; ++pc)
                w[mt * 3 + pc] = __builtin_bit_cast(bf16x8, ws[((REFIL_WSP_W1 + mt) * 6 + pc) * 64]);
        const Split3 xs = split3(xin[0], xin[1]);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            Split3 a;
            a.p[0] = w[mt * 3];
            a.p[1] = w[mt * 3 + 1];
            a.p[2] = w[mt * 3 + 2];
            x1[mt] = mfma_x6(a, xs, x1[mt]);
        }
    } else {
        mm_reg<4, KC1>(x1, P + L.w1, L.K1, 0, xin, lane);
    }
#else
    mm_reg<4, KC1>(x1, P + L.w1, L.K1, 0, xin, lane);
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i) x1[i] = relu4(x1[i]);
#if !defined(MLG_REFIL_INTRANS_F32)
    // in_trans as split-bf16 fp32 emulation (gru_tile_b16's scheme): x1 split once per 32-wide K step (K slot (g, i)
    // of step kk = the lane's own registers x1[2kk], x1[2kk + 1]), the weights pre-split in that K order (packed
    // section wsp), streamed in stages of 3 output tiles with the next stage's 18 loads issued before the current
    // stage's MFMAs. Tiles 0-3 = q (agent rows only), 4-11 = k | v. 144 bf16 MFMAs instead of 192 f32 MFMAs.
    (void)win;
    (void)ldin;
    {
        Split3 xs[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) xs[kk] = split3(x1[2 * kk], x1[2 * kk + 1]);
        const u32x4* ws = reinterpret_cast<const u32x4*>(P + L.wsp) + lane;
        bf16x8 wb[2][18];  // [tile in stage * 6 + kk * 3 + piece]
        auto load = [&](int stg, bf16x8 (&w)[18]) {
#pragma unroll
            for (int i = 0; i < 18; ++i) w[i] = __builtin_bit_cast(bf16x8, ws[(stg * 18 + i) * 64]);
        };
        load(0, wb[0]);
#pragma unroll
        for (int stg = 0; stg < 4; ++stg) {
            if (stg + 1 < 4) load(stg + 1, wb[(stg + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            const bf16x8(&w)[18] = wb[stg & 1];
#pragma unroll
            for (int ti = 0; ti < 3; ++ti) {
                const int mt = stg * 3 + ti;
                floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    Split3 a;
                    a.p[0] = w[ti * 6 + kk * 3 + 0];
                    a.p[1] = w[ti * 6 + kk * 3 + 1];
                    a.p[2] = w[ti * 6 + kk * 3 + 2];
                    acc = mfma_x6(a, xs[kk], acc);
                }
                if (mt < 4) {
                    if (col < NAS) st_row(qs, LDX, mt, acc, lane);
                } else {
                    st_row(kvs, LDKV, mt - 4, acc, lane);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#else
    {  // q: only the agent rows are queried
        floatx4 acc[4];
        bias_init<4>(acc, nullptr, 0, lane);
        mm_reg<4, 4>(acc, win, ldin, 0, x1, lane);
        if (col < NAS) {
#pragma unroll
            for (int i = 0; i < 4; ++i) st_row(qs, LDX, i, acc[i], lane);
        }
    }
#pragma unroll
    for (int m0 = 4; m0 < 12; m0 += 4) {  // k, v
        floatx4 acc[4];
        bias_init<4>(acc, nullptr, 0, lane);
        mm_reg<4, 4>(acc, win, ldin, m0, x1, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) st_row(kvs, LDKV, m0 - 4 + i, acc[i], lane);
    }
#endif
    wave_sync();
    if (nq <= 8)
        attn_fwd_half(qs, LDX, kvs, kvs + EMB, LDKV, mrow, nq, ne, o, LDX, lane);
    else
        attn_fwd_split(qs, LDX, kvs, kvs + EMB, LDKV, mrow, nq, ne, o, LDX, nullptr, lane);
    wave_sync();
}

// out_trans (+ post mask) -> fc2 -> ReLU -> GRUCell on the 16-row tile; h in/out (D layout).
// dead: bit r set = tile row r is a masked agent (post_mask, attention.py:75-76). wout / w2 may live in LDS (ld).
__device__ inline void agent_tile_post_w(const float* __restrict__ P, const RAgent& L, const float* wout, int ldo,
                                         const float* w2, int ld2, const float* o, uint32_t dead, floatx4 (&h)[4],
                                         int lane) {
    const int col = lane & 15;
    floatx4 x2[4], x3[4];
    bias_init<4>(x2, P + L.bout, 0, lane);
    mm_lds<4>(x2, wout, ldo, 0, o, LDX, EMB / 16, lane);
    if ((dead >> col) & 1u) {
#pragma unroll
        for (int i = 0; i < 4; ++i) x2[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    bias_init<4>(x3, P + L.b2, 0, lane);
    mm_reg<4, 4>(x3, w2, ld2, 0, x2, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) x3[i] = relu4(x3[i]);
#if defined(MLG_REFIL_GRU_PLAIN)
    gru_tile(P + L.wih, P + L.whh, P + L.bih, P + L.bhh, P + L.brz, x3, h, lane);
#elif defined(MLG_REFIL_GRU_F32)  // A/B: f32 MFMA products (round 1)
    gru_tile_pipe(P + L.wih, P + L.whh, P + L.bih, P + L.bhh, P + L.brz, x3, h, lane);
#else
    gru_tile_b16(P, L, x3, h, lane);
#endif
}

// Rollout form of agent_tile_post_w with out_trans and fc2 as split-bf16 fp32 emulation: o (LDS rows) is split once
// per 32-wide K step in the wsp K order (lane (col, g) reads features (2kk) * 16 + 4g .. + 3 and (2kk + 1) * 16 + 4g
// .. + 3 of row col), x2 from its D-layout registers; weights from the wsp tiles 12-19, all 48 loads issued up front.
__device__ inline void agent_tile_post_b16(const float* __restrict__ P, const RAgent& L, const float* o, uint32_t dead,
                                           floatx4 (&h)[4], int lane) {
    const int col = lane & 15, g = lane >> 4;
    const u32x4* ws = reinterpret_cast<const u32x4*>(P + L.wsp) + lane;
    bf16x8 wo[24], w2[24];  // [tile * 6 + kk * 3 + piece]
#pragma unroll
    for (int i = 0; i < 24; ++i) wo[i] = __builtin_bit_cast(bf16x8, ws[(REFIL_WSP_WOUT * 6 + i) * 64]);
    Split3 os[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
        os[kk] = split3(ld4(o + col * LDX + 2 * kk * 16 + 4 * g), ld4(o + col * LDX + (2 * kk + 1) * 16 + 4 * g));
    auto piece3 = [](const bf16x8 (&w)[24], int b) {
        Split3 s;
        s.p[0] = w[b];
        s.p[1] = w[b + 1];
        s.p[2] = w[b + 2];
        return s;
    };
    floatx4 x2[4], x3[4];
    bias_init<4>(x2, P + L.bout, 0, lane);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) x2[mt] = mfma_x6(piece3(wo, mt * 6 + kk * 3), os[kk], x2[mt]);
    // fc2's weights after out_trans' MFMAs are issued (wo's registers are free again: lower peak pressure)
#pragma unroll
    for (int i = 0; i < 24; ++i) w2[i] = __builtin_bit_cast(bf16x8, ws[(REFIL_WSP_W2 * 6 + i) * 64]);
    if ((dead >> col) & 1u) {
#pragma unroll
        for (int i = 0; i < 4; ++i) x2[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    Split3 xs[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) xs[kk] = split3(x2[2 * kk], x2[2 * kk + 1]);
    bias_init<4>(x3, P + L.b2, 0, lane);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) x3[mt] = mfma_x6(piece3(w2, mt * 6 + kk * 3), xs[kk], x3[mt]);
#pragma unroll
    for (int i = 0; i < 4; ++i) x3[i] = relu4(x3[i]);
    gru_tile_b16(P, L, x3, h, lane);
}

RO_PHASE void agent_tile_post(const float* __restrict__ P, const RAgent& L, const float* o, uint32_t dead,
                              floatx4 (&h)[4], int lane) {
    agent_tile_post_w(P, L, P + L.wout, EMB, P + L.w2, EMB, o, dead, h, lane);
}

// fc3 action tile `at` of the tile rows (q masked to 0 for dead rows, entity_rnn_agent.py:61)
__device__ __forceinline__ floatx4 agent_q(const float* __restrict__ P, const RAgent& L, const floatx4 (&h)[4], int at,
                                           uint32_t dead, int lane) {
    floatx4 q[1];
    bias_init<1>(q, P + L.b3, at, lane);
    mm_reg<1, 4>(q, P + L.w3, EMB, at, h, lane);
    if ((dead >> (lane & 15)) & 1u) q[0] = floatx4{0.f, 0.f, 0.f, 0.f};
    return q[0];
}

// ---- rollout ------------------------------------------------------------------------------------------------
struct RoLds {
    float q[NAS * LDX];
    float kv[NE * LDKV];
    float o[16 * LDX];
    float feat[2][NE][8];
    uint32_t om[2][NE];
    uint32_t em[2];
    uint32_t av[2][NAS];
    int x[2][NE], y[2][NE], hp[2][NE], act[2][NE], nhp[2][NE];
    int pk[2][NE];  // packed unit states x | y << 8 | hp << 16 (register env rules)
    int pact[2][NAS];
    int team[NE], role[NE], melee[NE], agent[NE];
    int status[2], len[2], slot[2], stepped[2];
    uint32_t ep[2];
    float ret[2];
};

struct RoArgs {
    int U, NA, A, ED, S, kmin, kmax, B;
    float inv_p;
};

__device__ __forceinline__ int64_t ro_slot(const MlgEntityBatch& bt, int b) {
    return bt.ring_size > 0 ? (int64_t)((bt.ring_slot0 + b) % bt.ring_size) : (int64_t)b;
}

// pre-transition data of step t for env e (lanes (e, u)); writes batch rows and the LDS copies
RO_PHASE void ro_observe(RoLds& S, const EnvTables& T, const EnvMasks& M, const RoArgs& a, const MlgEntityBatch& bt,
                         int e, int u, bool active, int t) {
    const bool me = active && u < a.U;
    // obs-mask and target bits of unit u, the units j split between the two half-waves (lanes 32-63 mirror unit u
    // of env e and scan j = 8..15) and ORed together by a permlane32 swap (all 64 lanes take part)
    uint32_t om_all, tb_all;
    {
        int pk[16];
        load16(S.pk[e], pk);
        const int pu = S.pk[e][u];
        const bool upper = (threadIdx.x & 32) != 0;
        const int xu = pkx(pu), yu = pky(pu);
        uint32_t om = 0u, tb, kb, ka, ke;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = (upper ? 8 : 0) + k;
            const int p = upper ? pk[8 + k] : pk[k];
            const int dx = pkx(p) - xu, dy = pky(p) - yu;
            om |= (uint32_t)(j < M.U && (pkh(p) <= 0 || dx * dx + dy * dy > MLG_SIGHT2)) << j;
        }
        unit_scan<8>(M, pk, u, pu, upper, tb, kb, ka, ke);
        const auto so = __builtin_amdgcn_permlane32_swap(om, om, false, false);
        const auto st = __builtin_amdgcn_permlane32_swap(tb, tb, false, false);
        om_all = om | (upper ? so[0] : so[1]);
        tb_all = tb | (upper ? st[0] : st[1]);
        if (pkh(pu) <= 0) om_all = (1u << M.U) - 1u;  // om_bits: a dead unit sees nothing
    }
    if (me) {
        const int pu = S.pk[e][u];
        const int64_t row = (S.slot[e] * (int64_t)bt.T1 + t);
        float f[8];
        entity_feat(T, pkx(pu), pky(pu), pkh(pu), u, a.inv_p, f);
        float* eg = bt.entities + (row * a.U + u) * a.ED;
        for (int k = 0; k < 8; ++k) {
            S.feat[e][u][k] = f[k];
            if (k < a.ED) eg[k] = f[k];
        }
        const uint32_t bits = om_all;
        uint8_t* omg = bt.obs_mask + (row * a.U + u) * a.U;
        if (a.U == 16) {  // one 16-byte row (rows of U bytes: 16-byte aligned when U == 16)
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                w[q] = ((bits >> (4 * q)) & 1u) | (((bits >> (4 * q + 1)) & 1u) << 8) |
                       (((bits >> (4 * q + 2)) & 1u) << 16) | (((bits >> (4 * q + 3)) & 1u) << 24);
            *reinterpret_cast<uint4*>(omg) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
            for (int j = 0; j < a.U; ++j) omg[j] = (uint8_t)((bits >> j) & 1u);
        }
        S.om[e][u] = bits;
        bt.entity_mask[row * a.U + u] = (uint8_t)(pkh(pu) <= 0);
        if (u < a.NA) {
            const uint32_t av = pkh(pu) <= 0 ? 1u
                                             : (((uint32_t)(pky(pu) + 1 < M.grid) << 1) | ((uint32_t)(pky(pu) - 1 >= 0) << 2) |
                                                ((uint32_t)(pkx(pu) + 1 < M.grid) << 3) | ((uint32_t)(pkx(pu) - 1 >= 0) << 4) |
                                                (tb_all << MLG_ACT_BASE));
            int32_t* ag = bt.avail + (row * a.NA + u) * a.A;
            for (int k = 0; k < a.A; ++k) ag[k] = (int)((av >> k) & 1u);
            S.av[e][u] = av;
        }
        if (u == 0) bt.filled[row] = 1;
    }
    const uint64_t bal = __ballot(me && pkh(S.pk[e][u]) <= 0);
    if (active && u == 0) S.em[e] = (uint32_t)((bal >> (16 * e)) & 0xFFFFu);
}

// zero bytes [b0, b1) of base with all 64 lanes: 16-byte stores for the aligned middle, byte stores at the edges
__device__ inline void zero_bytes(void* base, int64_t b0, int64_t b1, int lane) {
    if (b1 <= b0) return;
    uint8_t* p = reinterpret_cast<uint8_t*>(base);
    const uintptr_t ua = ((uintptr_t)(p + b0) + 15) & ~(uintptr_t)15, ub = (uintptr_t)(p + b1) & ~(uintptr_t)15;
    int64_t m0 = (int64_t)(ua - (uintptr_t)p), m1 = (int64_t)(ub - (uintptr_t)p);
    if (m0 > b1 || m1 < m0) m0 = m1 = b1;  // too short for an aligned middle
    for (int64_t i = b0 + lane; i < m0; i += 64) p[i] = 0;
    for (int64_t i = m0 + 16 * (int64_t)lane; i < m1; i += 16 * 64) *reinterpret_cast<uint4*>(p + i) = make_uint4(0, 0, 0, 0);
    for (int64_t i = (m1 > b0 ? m1 : b0) + lane; i < b1; i += 64) p[i] = 0;
}

// zero rows [t0, end) of every key of slot `slot` (full-write ring mode), all 64 lanes; end = T1, or the slot's
// extent (MlgEntityBatch.slot_extent: the rows of its previous episode that may be non-zero), which then becomes t0
__device__ inline void ro_zero_tail(const MlgEntityBatch& bt, const RoArgs& a, int64_t slot, int t0, int lane) {
    int end = bt.T1;
    if (bt.slot_extent) {
        const int x = bt.slot_extent[slot];
        end = x < 0 ? 0 : (x < bt.T1 ? x : bt.T1);
    }
    // the new extent is stored once `end` is known (the old value has been read by every lane)
    if (bt.slot_extent && lane == 0) bt.slot_extent[slot] = t0;
    if (t0 >= end) return;
    const int64_t r0 = slot * bt.T1 + t0, r1 = slot * (int64_t)bt.T1 + end;
    auto z = [&](void* p, int64_t row_bytes) { zero_bytes(p, r0 * row_bytes, r1 * row_bytes, lane); };
    z(bt.entities, (int64_t)a.U * a.ED * 4);
    z(bt.actions_onehot, (int64_t)a.NA * a.A * 4);
    z(bt.reward, 4);
    z(bt.obs_mask, (int64_t)a.U * a.U);
    z(bt.entity_mask, a.U);
    z(bt.actions, (int64_t)a.NA * 8);
    z(bt.avail, (int64_t)a.NA * a.A * 4);
    z(bt.terminated, 1);
    z(bt.filled, 8);
}

// Workgroup = RO_WAVES waves; every wave owns two envs for the whole episode (no cross-wave dependency after the
// prologue); the waves share one LDS copy of in_trans / out_trans / fc2 (padded rows, conflict-free A reads).
constexpr int RO_WAVES = 4;
constexpr int LDW = EMB + 4;
// fp32 in_trans / out_trans / fc2 copies in LDS only for the f32 A/B forms; the split-bf16 default streams the
// pre-split weights from L2 (69 KB of LDS per workgroup instead of 156 KB)
#if defined(MLG_REFIL_INTRANS_F32) || defined(MLG_REFIL_POST_F32) || defined(MLG_REFIL_GRU_PLAIN) || defined(MLG_REFIL_GRU_F32)
#define RO_LDS_WEIGHTS 1
#endif
struct RoShared {
#ifdef RO_LDS_WEIGHTS
    float win[3 * EMB * LDW];
    float wout[EMB * LDW];
    float w2[EMB * LDW];
#endif
    RoLds S[RO_WAVES];
};

template <int KC1>
#ifdef MLG_REFIL_W2  // experiment: two waves per SIMD (<= 256 VGPR + AGPR per lane)
#define RO_OCC __attribute__((amdgpu_waves_per_eu(2, 2)))
#else
#define RO_OCC
#endif
__global__ void __launch_bounds__(64 * RO_WAVES) RO_OCC refil_rollout_kernel(MlgEntityEnvSpec spec, MlgEnvState st, RAgent L,
                                                                      const float* __restrict__ P, MlgEntityBatch bt,
                                                                      MlgRunInfo info, RoArgs a, float eps,
                                                                      int test_mode) {
    extern __shared__ __attribute__((aligned(16))) float ro_smem[];
    RoShared& SH = *reinterpret_cast<RoShared*>(ro_smem);
#ifdef RO_LDS_WEIGHTS
    for (int i = threadIdx.x; i < 3 * EMB * EMB; i += blockDim.x) SH.win[(i / EMB) * LDW + i % EMB] = P[L.win + i];
    for (int i = threadIdx.x; i < EMB * EMB; i += blockDim.x) {
        SH.wout[(i / EMB) * LDW + i % EMB] = P[L.wout + i];
        SH.w2[(i / EMB) * LDW + i % EMB] = P[L.w2 + i];
    }
    const float* sh_win = SH.win;
#else
    const float* sh_win = nullptr;
#endif
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    RoLds& S = SH.S[wave];
    RStamps stp;
    stp.init();
    const int lane = threadIdx.x & 63;
    const int e = (lane >> 4) & 1, u = lane & 15;
    const bool env_lane = lane < 32;
    const int b0 = (blockIdx.x * RO_WAVES + wave) * 2;
    const MlgEnvSpec& sp = spec.base;
    if (lane < a.U) {
        S.team[lane] = sp.team[lane];
        S.role[lane] = sp.role[lane];
        S.melee[lane] = sp.melee[lane];
        S.agent[lane] = lane < a.NA ? lane + 1 : 0;
    }
    for (int i = lane; i < 16 * LDX; i += 64) S.o[i] = 0.f;
    if (lane < 2) {
        const int b = b0 + lane;
        S.status[lane] = b < a.B ? 0 : 2;
        S.len[lane] = 0;
        S.ret[lane] = 0.f;
        S.stepped[lane] = 0;
        S.slot[lane] = b < a.B ? (int)ro_slot(bt, b) : 0;
        S.ep[lane] = b < a.B ? st.episode[b] : 0u;
    }
    if (lane < 16) S.pact[lane >> 3][lane & 7] = 0;
    wave_sync();
    EnvTables T;
    T.team = S.team;
    T.role = S.role;
    T.melee = S.melee;
    T.agent = S.agent;
    T.U = a.U;
    T.grid = sp.grid;
    T.episode_limit = sp.episode_limit;
    T.stochastic = sp.stochastic;
    EnvMasks M;
    M.team1 = M.healer = M.tank = M.melee = 0;
    for (int j = 0; j < a.U; ++j) {
        M.team1 |= (uint32_t)(S.team[j] != 0) << j;
        M.healer |= (uint32_t)(S.role[j] == 1) << j;
        M.tank |= (uint32_t)(S.role[j] == 0) << j;
        M.melee |= (uint32_t)(S.melee[j] != 0) << j;
    }
    M.U = a.U;
    M.grid = sp.grid;
    // ---- reset (EnvWorker "reset", env_worker_process.py:54-60) ----
    const int b = b0 + e;
    const bool live = env_lane && b < a.B;
    if (live && u < a.U) {
        const uint64_t key = mlg_env_key(sp.seed, b);
        const uint32_t ep = S.ep[e];
        const int k = entity_team_k(key, ep, a.kmin, a.kmax);
        const int tf = S.team[u] ? a.S : 0;
        int xx, yy, hh;
        env_spawn_xyh(T, key, ep, u, tf, a.S, xx, yy, hh);
        if (u - tf >= k) hh = 0;
        S.x[e][u] = xx;
        S.y[e][u] = yy;
        S.hp[e][u] = hh;
        S.pk[e][u] = pk_pack(xx, yy, hh);
    }
    if (env_lane && u >= a.U) S.pk[e][u] = 0;
    wave_sync();
    ro_observe(S, T, M, a, bt, e, u, live, 0);
    wave_sync();
    floatx4 h[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    uint64_t rows = 0;
    const int col = lane & 15, g = lane >> 4;
    for (int t = 0;; ++t) {
        const int st0 = S.status[0], st1 = S.status[1];
        if (st0 == 2 && st1 == 2) break;
        // opaque per-iteration copy of the weight pointer: keeps the compiler from hoisting every (loop-invariant)
        // weight load of the step out of the episode loop into registers (> 512 VGPRs, spills)
        int64_t zoff = 0;
        asm volatile("" : "+s"(zoff));
        const float* __restrict__ Pw = P + zoff;
        // ---- agent phase: EntityMAC.forward(t) + epsilon-greedy for both envs ----
        for (int ee = 0; ee < 2; ++ee) {
            if (S.status[ee] == 2) continue;
            // fc1 B operand: lane (entity j = col, g) holds inputs k = 16 kc + 4 g + r
            floatx4 xin[KC1];
            const int j = col;
#pragma unroll
            for (int kc = 0; kc < KC1; ++kc)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int k = kc * 16 + 4 * g + r;
                    float v = 0.f;
                    if (j < a.U) {
                        if (k < a.ED) v = S.feat[ee][j][k < 8 ? k : 0];
                        else if (k < a.ED + a.A && j < a.NA && t > 0 && S.pact[ee][j] == k - a.ED) v = 1.f;
                    }
                    xin[kc][r] = v;
                }
            stp.mark(0);
            entity_block_reg<KC1>(Pw, L, sh_win, LDW, xin, S.q, S.kv, S.om[ee], a.NA, a.U, S.o + ee * NAS * LDX, lane);
            stp.mark(1);
            rows += (uint64_t)a.NA;
        }
        // tile row r = env (r >> 3), agent (r & 7); dead = agent entity masked
        uint32_t dead = 0;
        for (int ee = 0; ee < 2; ++ee) {
            uint32_t m = S.em[ee] & ((1u << a.NA) - 1u);
            m |= ~((1u << a.NA) - 1u) & 0xFFu;  // padding rows >= n_agents
            dead |= (m & 0xFFu) << (8 * ee);
        }
#if defined(MLG_REFIL_POST_F32) || defined(MLG_REFIL_GRU_PLAIN) || defined(MLG_REFIL_GRU_F32)
        agent_tile_post_w(Pw, L, SH.wout, LDW, SH.w2, LDW, S.o, dead, h, lane);
#else
        agent_tile_post_b16(Pw, L, S.o, dead, h, lane);
#endif
        stp.mark(2);
        // fc3 + masked argmax + epsilon-greedy
        const int re = col >> 3, rn = col & 7;
        const uint32_t avm = (rn < a.NA) ? S.av[re][rn] : 1u;
        ArgmaxState as{-INFINITY, 1 << 30};
#if !defined(MLG_REFIL_POST_F32) && !defined(MLG_REFIL_GRU_PLAIN) && !defined(MLG_REFIL_GRU_F32)
        Split3 hs3[2];  // fc3 as split-bf16 (wsp tiles 24-25; Ap <= 32 host-checked)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) hs3[kk] = split3(h[2 * kk], h[2 * kk + 1]);
#endif
        for (int at = 0; at < L.Ap / 16; ++at) {
#if !defined(MLG_REFIL_POST_F32) && !defined(MLG_REFIL_GRU_PLAIN) && !defined(MLG_REFIL_GRU_F32)
            floatx4 q;
            {
                const u32x4* ws = reinterpret_cast<const u32x4*>(Pw + L.wsp) + lane;
                bf16x8 w[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) w[i] = __builtin_bit_cast(bf16x8, ws[((REFIL_WSP_W3 + at) * 6 + i) * 64]);
                q = ld4(Pw + L.b3 + at * 16 + 4 * g);
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    Split3 a3;
                    a3.p[0] = w[kk * 3];
                    a3.p[1] = w[kk * 3 + 1];
                    a3.p[2] = w[kk * 3 + 2];
                    q = mfma_x6(a3, hs3[kk], q);
                }
                if ((dead >> (lane & 15)) & 1u) q = floatx4{0.f, 0.f, 0.f, 0.f};
            }
#else
            const floatx4 q = agent_q(Pw, L, h, at, dead, lane);
#endif
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ac = at * 16 + 4 * g + r;
                if (ac >= a.A) continue;
                const float v = ((avm >> ac) & 1u) ? q[r] : -INFINITY;
                if (amax_better(v, ac, as.bv, as.bi)) { as.bv = v; as.bi = ac; }
            }
        }
        int act = argmax_reduce(as);
        const int bb = b0 + re;
        if (g == 0 && rn < a.NA && S.status[re] != 2) {
            if (!test_mode && eps > 0.f) {
                const uint64_t key = mlg_env_key(sp.seed, bb);
                const uint64_t r1 = mlg_rng(key, mlg_ctr(S.ep[re], (uint32_t)t, MLG_PURPOSE_EPS, (uint32_t)rn));
                if (mlg_u01(r1) < eps) {
                    const uint64_t r2 = mlg_rng(key, mlg_ctr(S.ep[re], (uint32_t)t, MLG_PURPOSE_RAND, (uint32_t)rn));
                    const int na = __popc(avm);
                    if (na == 0) {
                        act = 0;
                    } else {
                        const int k = (int)(((r2 >> 40) * (uint64_t)na) >> 24);
                        uint32_t m = avm;
                        for (int i = 0; i < k; ++i) m &= m - 1;
                        act = __ffs((int)m) - 1;
                    }
                }
            }
            S.pact[re][rn] = act;
            const int64_t off = ((int64_t)S.slot[re] * bt.T1 + t) * a.NA + rn;
            bt.actions[off] = act;
            float* oh = bt.actions_onehot + off * a.A;
            if (bt.full_write) {
                for (int k = 0; k < a.A; ++k) oh[k] = k == act ? 1.f : 0.f;
            } else {
                oh[act] = 1.f;
            }
        }
        wave_sync();
        stp.mark(3);
        // ---- env phase (EnvWorker "step", env_worker_process.py:32-53) ----
        const bool stepping = env_lane && S.status[e] == 0;
        int pk[16];
        load16(S.pk[e], pk);
        const int pu = S.pk[e][u];
        {  // executed action: validated policy action or scripted AI (spec §3.4). Lanes 32-63 (no env of their
           // own) mirror unit u of env e and scan the upper half of the units j; partials combine by permlane32
            uint32_t tb, kb, ka, ke;
            unit_scan<8>(M, pk, u, pu, lane >= 32, tb, kb, ka, ke);
            auto other = [](uint32_t v) {  // lane l ^ 32
                const auto s2 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
                return (threadIdx.x & 32) ? s2[0] : s2[1];
            };
            tb |= other(tb);
            kb = min(kb, other(kb));
            ka = min(ka, other(ka));
            ke = min(ke, other(ke));
            if (stepping && u < a.U) {
                int ac;
                if (u < a.NA) {
                    const int pa = S.pact[e][u];
                    const uint32_t av = pkh(pu) <= 0 ? 1u
                                                     : (((uint32_t)(pky(pu) + 1 < M.grid) << 1) |
                                                        ((uint32_t)(pky(pu) - 1 >= 0) << 2) |
                                                        ((uint32_t)(pkx(pu) + 1 < M.grid) << 3) |
                                                        ((uint32_t)(pkx(pu) - 1 >= 0) << 4) | (tb << MLG_ACT_BASE));
                    ac = (pa >= 0 && pa < MLG_ACT_BASE + a.U && ((av >> pa) & 1u)) ? pa : 0;
                } else {
                    ac = ai_from_scan(M, u, pu, kb, ka, ke, [&](int j) { return S.pk[e][j]; });
                }
                S.act[e][u] = ac;
            }
        }
        wave_sync();
        stp.mark(4);
        if (stepping && u < a.U) {
            int acts[16];
            load16(S.act[e], acts);
            S.nhp[e][u] = resolve_hp_reg(M, pk, acts, u, pu);
        }
        wave_sync();
        stp.mark(5);
        if (stepping && u < a.U && S.hp[e][u] > 0) env_apply_move(S.act[e][u], &S.x[e][u], &S.y[e][u]);
        // per-unit step results as lane ballots (bit 16 e + u): alive after, killed, bits of the hp lost (<= 64);
        // the reward below counts them per team instead of a serial loop over the units in one lane
        uint64_t rw_alive, rw_kill, rw_loss[7];
        {
            const bool v = stepping && u < a.U;
            const int h0 = v ? S.hp[e][u] : 0, h1 = v ? S.nhp[e][u] : 0;
            const int loss = (h0 > 0 && h0 > h1) ? h0 - h1 : 0;
            rw_alive = __ballot(v && h1 > 0);
            rw_kill = __ballot(v && h0 > 0 && h1 == 0);
#pragma unroll
            for (int bb = 0; bb < 7; ++bb) rw_loss[bb] = __ballot((loss >> bb) & 1);
        }
        if (env_lane && u == 0) {
            const int stt = S.status[e];
            S.stepped[e] = 0;
            const int64_t sl = (int64_t)S.slot[e] * bt.T1 + t;
            if (stt == 1) {  // final action recorded (parallel_stepper.py:153); env done
                S.status[e] = 2;
                if (bt.full_write) {
                    bt.reward[sl] = 0.f;
                    bt.terminated[sl] = 0;
                }
            } else if (stt == 0) {
                int alive[2] = {0, 0}, lost[2] = {0, 0}, kills[2] = {0, 0};
                const uint32_t t1 = M.team1 & ((1u << a.U) - 1u);
                const uint32_t am = (uint32_t)(rw_alive >> (16 * e)) & 0xFFFFu, km = (uint32_t)(rw_kill >> (16 * e)) & 0xFFFFu;
                alive[0] = __builtin_popcount(am & ~t1);
                alive[1] = __builtin_popcount(am & t1);
                kills[0] = __builtin_popcount(km & t1);  // team-1 units killed: credited to team 0
                kills[1] = __builtin_popcount(km & ~t1);
#pragma unroll
                for (int bb = 0; bb < 7; ++bb) {
                    const uint32_t lm = (uint32_t)(rw_loss[bb] >> (16 * e)) & 0xFFFFu;
                    lost[0] += __builtin_popcount(lm & ~t1) << bb;
                    lost[1] += __builtin_popcount(lm & t1) << bb;
                }
                const int done = alive[0] == 0 || alive[1] == 0 || t + 1 >= sp.episode_limit;
                const int w0 = alive[1] == 0 && alive[0] > 0, w1 = alive[0] == 0 && alive[1] > 0;
                const float r = (float)(lost[1] + 10 * kills[0] + 200 * w0) * 0.0625f;  // policy team 0
                bt.reward[sl] = r;
                bt.terminated[sl] = (uint8_t)done;
                S.ret[e] += r;
                S.stepped[e] = 1;
                if (done) {
                    S.status[e] = 1;
                    S.len[e] = t + 1;
                    const int bb2 = b0 + e;
                    info.won[2 * bb2] = w0;
                    info.won[2 * bb2 + 1] = w1;
                    info.draw[bb2] = !w0 && !w1;
                }
            }
        }
        wave_sync();
        stp.mark(6);
        const bool stepped = env_lane && S.stepped[e];
        if (stepped && u < a.U) {
            S.hp[e][u] = S.nhp[e][u];
            S.pk[e][u] = pk_pack(S.x[e][u], S.y[e][u], S.nhp[e][u]);
        }
        wave_sync();
        ro_observe(S, T, M, a, bt, e, u, stepped, t + 1);
        wave_sync();
        stp.mark(7);
    }
    // ---- finish: run summary, env state, full-write tails ----
    if (live && u == 0) {
        info.ep_len[b] = S.len[e];
        info.ret[b] = S.ret[e];
        st.t[b] = S.len[e];
        st.episode[b] = S.ep[e] + 1u;
    }
    if (live && u < a.U) {
        st.x[(int64_t)b * a.U + u] = S.x[e][u];
        st.y[(int64_t)b * a.U + u] = S.y[e][u];
        st.hp[(int64_t)b * a.U + u] = S.hp[e][u];
    }
    if (bt.full_write) {
        for (int ee = 0; ee < 2; ++ee)
            if (b0 + ee < a.B) ro_zero_tail(bt, a, S.slot[ee], S.len[ee] + 1, lane);
    }
    if (info.agent_rows && lane == 0) atomicAdd((unsigned long long*)info.agent_rows, (unsigned long long)rows);
    stp.mark(8);
    stp.flush();
}

// ---- one EntityAttentionRNNAgent step over R items (two items per wave) -------------------------------
__global__ void __launch_bounds__(64) refil_agent_step_kernel(RAgent L, const float* __restrict__ P, int R, int NA,
                                                              int NEa, int D0, int A, const float* __restrict__ ent,
                                                              const uint8_t* __restrict__ om,
                                                              const uint8_t* __restrict__ em,
                                                              const float* __restrict__ h_in, float* __restrict__ q_out,
                                                              float* __restrict__ h_out) {
    __shared__ float ein[NE * LDI];
    __shared__ float x1[NE * LDX];
    __shared__ float qkv[NE * LDQ];
    __shared__ float o[16 * LDX];
    __shared__ uint32_t mrow[2][NE];
    __shared__ uint32_t emb[2];
    const int lane = threadIdx.x;
    const int i0 = blockIdx.x * 2;
    for (int i = lane; i < 16 * LDX; i += 64) o[i] = 0.f;
    if (lane < 32) {
        const int e = lane >> 4, q = lane & 15;
        const int it = i0 + e;
        uint32_t bits = 0xFFFFFFFFu;
        if (it < R && q < NEa) {
            bits = 0;
            for (int j = 0; j < NEa; ++j) bits |= (uint32_t)(om[((int64_t)it * NEa + q) * NEa + j] != 0) << j;
        }
        mrow[e][q] = bits;
        if (q == 0) {
            uint32_t m = 0xFFFFFFFFu;
            if (it < R) {
                m = 0;
                for (int j = 0; j < NEa; ++j) m |= (uint32_t)(em[(int64_t)it * NEa + j] != 0) << j;
                m |= ~((1u << NEa) - 1u);
            }
            emb[e] = m;
        }
    }
    wave_sync();
    for (int e = 0; e < 2; ++e) {
        const int it = i0 + e;
        for (int i = lane; i < NE * L.K1; i += 64) {
            const int j = i / L.K1, c = i % L.K1;
            ein[j * LDI + c] = (it < R && j < NEa && c < D0) ? ent[((int64_t)it * NEa + j) * D0 + c] : 0.f;
        }
        wave_sync();
        entity_block(P, L, ein, x1, qkv, mrow[e], NA, NEa, o + e * NAS * LDX, lane);
    }
    const int col = lane & 15, g = lane >> 4;
    const int e = col >> 3, n = col & 7, it = i0 + e;
    const bool valid = it < R && n < NA;
    uint32_t dead = 0;
    for (int ee = 0; ee < 2; ++ee) dead |= ((emb[ee] | ~((1u << NA) - 1u)) & 0xFFu) << (8 * ee);
    floatx4 h[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
        h[mt] = valid ? ld4(h_in + ((int64_t)it * NA + n) * EMB + mt * 16 + 4 * g) : floatx4{0.f, 0.f, 0.f, 0.f};
    agent_tile_post(P, L, o, dead, h, lane);
    if (valid) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) *reinterpret_cast<floatx4*>(h_out + ((int64_t)it * NA + n) * EMB + mt * 16 + 4 * g) = h[mt];
    }
    for (int at = 0; at < L.Ap / 16; ++at) {
        const floatx4 q = agent_q(P, L, h, at, dead, lane);
        if (valid) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ac = at * 16 + 4 * g + r;
                if (ac < A) q_out[((int64_t)it * NA + n) * A + ac] = q[r];
            }
        }
    }
}

#include "refil_ro4.inc"

}  // namespace

extern "C" int mlg_refil_debug_set_stamps(void* ptr) {
#ifdef MLG_STAMPS
    unsigned long long* p = (unsigned long long*)ptr;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_refil_stamps), &p, sizeof(p)) != hipSuccess) return mlg::fail("set stamps");
    return 0;
#else
    (void)ptr;
    return mlg::fail("mlg_refil_debug_set_stamps: build with -DMLG_STAMPS (make stamps)");
#endif
}

extern "C" int64_t mlg_refil_packed_agent_size(const MlgRefilDims* d) {
    if (check_dims(d)) return -1;
    return agent_layout(d).total;
}

extern "C" int mlg_refil_pack_agent(const MlgRefilDims* d, const float* flat, float* packed, void* stream) {
    if (check_dims(d)) return 1;
    MLG_REQUIRE(flat && packed, "refil_pack_agent: null pointer");
    const RAgent L = agent_layout(d);
    if (launch_copy(agent_pack_jobs(L), flat, packed, (hipStream_t)stream)) return 1;
    hipLaunchKernelGGL(refil_pack_gsp_kernel, dim3((unsigned)((REFIL_GSP + REFIL_WSP + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream,
                       L, flat, packed);
    return mlg::check_launch("refil_pack_gsp_kernel");
}

extern "C" int mlg_refil_agent_forward(const MlgRefilDims* d, const float* packed, const float* entities,
                                       const uint8_t* obs_mask, const uint8_t* entity_mask, const float* h_in, float* q,
                                       float* h_out, int32_t R, void* stream) {
    if (check_dims(d)) return 1;
    MLG_REQUIRE(packed && entities && obs_mask && entity_mask && h_in && q && h_out, "refil_agent_forward: null pointer");
    MLG_REQUIRE(R >= 0, "refil_agent_forward: R=%d", R);
    if (R == 0) return 0;
    const RAgent L = agent_layout(d);
    hipLaunchKernelGGL(refil_agent_step_kernel, dim3((unsigned)((R + 1) / 2)), dim3(64), 0, (hipStream_t)stream, L, packed,
                       R, d->n_agents, d->n_entities, L.D0, d->n_actions, entities, obs_mask, entity_mask, h_in, q, h_out);
    return mlg::check_launch("refil_agent_forward");
}

extern "C" int mlg_refil_rollout(const MlgEntityEnvSpec* spec, MlgEnvState* st, const MlgRefilDims* d,
                                 const float* packed, MlgEntityBatch* batch, MlgRunInfo* info, float epsilon,
                                 int32_t test_mode, void* stream) {
    if (check_dims(d)) return 1;
    MLG_REQUIRE(spec && st && packed && batch && info, "refil_rollout: null argument");
    const MlgEnvSpec& sp = spec->base;
    const int S = sp.U / 2;
    MLG_REQUIRE(sp.U % 2 == 0 && sp.U <= NE && S <= NAS, "refil_rollout: U=%d unsupported (even, <= 16)", sp.U);
    MLG_REQUIRE(sp.n_agents == S && d->n_agents == S && d->n_entities == sp.U && d->entity_shape == 8 &&
                    d->n_actions == MLG_ACT_BASE + sp.U && d->entity_last_action,
                "refil_rollout: dims (n_agents=%d n_entities=%d entity_shape=%d n_actions=%d) do not match the env "
                "(S=%d, U=%d)", d->n_agents, d->n_entities, d->entity_shape, d->n_actions, S, sp.U);
    MLG_REQUIRE(spec->min_agents >= 1 && spec->min_agents <= spec->max_agents && spec->max_agents <= S,
                "refil_rollout: min_agents=%d max_agents=%d (slots %d)", spec->min_agents, spec->max_agents, S);
    MLG_REQUIRE(sp.policy_team == 0 && sp.scripted[0] == 0 && sp.scripted[1] == 1,
                "refil_rollout: the entity env has policy team 0 and scripted team 1");
    const MlgEntityBatch& bt = *batch;
    MLG_REQUIRE(bt.entities && bt.obs_mask && bt.entity_mask && bt.actions && bt.avail && bt.reward && bt.terminated &&
                    bt.actions_onehot && bt.filled, "refil_rollout: batch has null tensors");
    MLG_REQUIRE(st->B == bt.B && bt.T1 >= sp.episode_limit + 1, "refil_rollout: B=%d/%d T1=%d (episode_limit %d)", st->B,
                bt.B, bt.T1, sp.episode_limit);
    MLG_REQUIRE(info->ep_len && info->ret && info->won && info->draw, "refil_rollout: run info has null buffers");
    if (bt.B == 0) return 0;
    int p = 1;
    while (p < sp.grid) p <<= 1;
    RoArgs a{sp.U, S, d->n_actions, d->entity_shape, S, spec->min_agents, spec->max_agents, bt.B, 1.0f / (float)p};
    const RAgent L = agent_layout(d);
    // default: four envs per wave (refil_ro4.inc) for the entity width of the env variant (K1 = 32);
    // MLG_REFIL_ROLLOUT=v1 selects the two-env kernel (A/B, parity tests run both)
    const char* var = getenv("MLG_REFIL_ROLLOUT");
    const bool v1 = (var && strcmp(var, "v1") == 0) || L.K1 != 32;
    if (!v1) {
        const size_t lds4 = sizeof(R4Shared);
        // the refil_8 shape (16 units: the checks above fix the rest of the dims) as the static instantiation
        // (MLG_REFIL_GENERIC=1: the generic one, A/B)
        const bool generic = getenv("MLG_REFIL_GENERIC") != nullptr;
        const bool st16 = sp.U == 16 && !generic;
        auto kern4 = st16 ? refil_rollout4_kernel<2, 16> : refil_rollout4_kernel<2, 0>;
        static bool attr4[2] = {false, false};
        if (!attr4[st16]) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern4),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds4);
            if (e != hipSuccess) return mlg::fail("refil_rollout: LDS %zu B: %s", lds4, hipGetErrorString(e));
            attr4[st16] = true;
        }
        const int per_block4 = R4_ENVS * R4_WAVES;
        hipLaunchKernelGGL(kern4, dim3((unsigned)((bt.B + per_block4 - 1) / per_block4)), dim3(64 * R4_WAVES), lds4,
                           (hipStream_t)stream, *spec, *st, L, packed, bt, *info, a, test_mode ? 0.f : epsilon,
                           test_mode);
        return mlg::check_launch("refil_rollout4");
    }
    auto kern = L.K1 <= 16 ? refil_rollout_kernel<1> : (L.K1 <= 32 ? refil_rollout_kernel<2> : refil_rollout_kernel<3>);
    const size_t lds = sizeof(RoShared);
    static bool attr_set[3] = {false, false, false};
    const int ki = L.K1 <= 16 ? 0 : (L.K1 <= 32 ? 1 : 2);
    if (!attr_set[ki]) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (e != hipSuccess) return mlg::fail("refil_rollout: LDS %zu B: %s", lds, hipGetErrorString(e));
        attr_set[ki] = true;
    }
    const int per_block = 2 * RO_WAVES;
    hipLaunchKernelGGL(kern, dim3((unsigned)((bt.B + per_block - 1) / per_block)), dim3(64 * RO_WAVES), lds,
                       (hipStream_t)stream, *spec, *st, L, packed, bt, *info, a, test_mode ? 0.f : epsilon, test_mode);
    return mlg::check_launch("refil_rollout");
}
