// mlg_device.h -- shared device helpers for the gfx950 kernels of libmaleague.
//
// * f32 MFMA (v_mfma_f32_16x16x4_f32) fragment helpers for the 16-row agent tiles
// * the counter-based RNG of the env spec (splitmix64)
// * the synthetic TeamsEnv spec v1 as device functions (bit-exact restatement checked against
//   oracle/env_ref.c; the reference env itself -- external maenv -- is not available)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/maleague.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define MLG_ACT_BASE 5
#define MLG_SIGHT2 36

// ------------------------------------------------------------------------------------------------
// MFMA: D[16x16] += A[16x4] * B[4x16]; lane l supplies A[l&15][l>>4], B[l>>4][l&15];
// D lane l, reg r = D[4*(l>>4)+r][l&15].  Orientation used everywhere below: A = weights
// (rows = output features), B = activations (cols = agent rows), so a result tile is already the
// B operand of the next layer with the K index permuted (feature 16c + 4*(l>>4) + r at step (c, r)),
// and the weight operand is read with the same permutation as one float4 per 4 MFMAs.
__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ floatx4 ld4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }
// Store through the global address space. A pointer whose provenance the compiler cannot see (kept in VGPRs behind
// an opaque asm, e.g. the rollout's per-step batch pointers) is otherwise stored through as FLAT: flat stores count
// on lgkmcnt too, so every later LDS / permute wait would also wait for the step's HBM stores to complete. Batch,
// run-summary (zero-copy host) and ring pointers are all global memory.
template <class T>
__device__ __forceinline__ void gst(T* p, T v) {
    *(__attribute__((address_space(1))) T*)p = v;
}
// HIP's struct vector types have no assignment into another address space: store their native vector form
__device__ __forceinline__ void gst(uint4* p, uint4 v) {
    typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
    gst(reinterpret_cast<u32x4_*>(p), u32x4_{v.x, v.y, v.z, v.w});
}
__device__ __forceinline__ void gst(float2* p, float2 v) {
    typedef float f32x2_ __attribute__((ext_vector_type(2)));
    gst(reinterpret_cast<f32x2_*>(p), f32x2_{v.x, v.y});
}

// bf16 operands of v_mfma_f32_16x16x32_bf16 (8 per lane) and round-to-nearest packing of two fp32 (low half = lo).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned int cvt_pk_bf16(float lo, float hi) {
    unsigned int r;
    asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
    return r;
}

__device__ __forceinline__ floatx4 mfma_bf16(bf16x8 a, bf16x8 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// GRU gates on the hardware exp / reciprocal (v_exp_f32, v_rcp_f32; ~1 ulp each) instead of libm expf / tanhf and
// IEEE division (~70 instructions with range branches): used by the v7 rollout and the learner recurrence, whose
// parity bars are tolerance-based (Q 1e-4, learner stats rtol 1e-4); tanh(x) = 2 sigmoid(2x) - 1.
__device__ __forceinline__ float fast_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float fast_tanh(float x) { return 2.f * fast_sigmoid(2.f * x) - 1.f; }

// ---- split-bf16 fp32 emulation pieces (shared by the rollout kernels) ----
struct Split3 {
    bf16x8 p[3];
};

// 8 fp32 -> three bf16x8 pieces (element j of every piece belongs to input j).
__device__ __forceinline__ Split3 split3(floatx4 a, floatx4 b) {
    float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    Split3 s;
#pragma unroll
    for (int lvl = 0; lvl < 3; ++lvl) {
        u32x4 w;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned int pk = cvt_pk_bf16(v[2 * q], v[2 * q + 1]);
            w[q] = pk;
            if (lvl < 2) {  // remainders (exact in fp32)
                v[2 * q] -= __uint_as_float(pk << 16);
                v[2 * q + 1] -= __uint_as_float(pk & 0xFFFF0000u);
            }
        }
        s.p[lvl] = __builtin_bit_cast(bf16x8, w);
    }
    return s;
}


// acc += A . B over one 32-wide K step with the six partial products (small terms first).
__device__ __forceinline__ floatx4 mfma_x6(const Split3& a, const Split3& b, floatx4 c) {
    c = mfma_bf16(a.p[2], b.p[0], c);
    c = mfma_bf16(a.p[1], b.p[1], c);
    c = mfma_bf16(a.p[0], b.p[2], c);
    c = mfma_bf16(a.p[1], b.p[0], c);
    c = mfma_bf16(a.p[0], b.p[1], c);
    c = mfma_bf16(a.p[0], b.p[0], c);
    return c;
}

// Piece `piece` (0..2) of the split-bf16 representation of the pair (a, b) as one u32 (bf16 of a low, of b high),
// bit-identical to split3() in rollout.hip: a = a0 + a1 + a2 exactly, round to nearest per piece.
__device__ __forceinline__ float split_bf16_pair(float a, float b, int piece) {
    unsigned int pk = 0u;
    for (int lvl = 0; lvl <= piece; ++lvl) {
        pk = cvt_pk_bf16(a, b);
        a -= __uint_as_float(pk << 16);
        b -= __uint_as_float(pk & 0xFFFF0000u);
    }
    return __uint_as_float(pk);
}

// Workgroup barrier that orders LDS only: the release fence waits for this wave's LDS operations (lgkmcnt) but not
// for its outstanding global stores, which __syncthreads() (a release fence over all address spaces) waits for --
// on the rollout's per-step barriers that was the HBM write latency of the step's action / batch-row stores. Only
// for kernels whose waves never read, within the kernel, global data another wave of the workgroup wrote (the
// rollout kernels: batch rows and actions are write-only there, cross-wave data goes through LDS).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Cross-lane reads without LDS (v_permlane16/32_swap, VALU): lane_plus16 returns lane l + 16's value in lanes of
// the even 16-lane rows (0..15, 32..47); lane_plus32 returns lane l + 32's value in lanes 0..31. Other lanes get
// unspecified values.
__device__ __forceinline__ float lane_plus16(float x) {
    const unsigned u = __float_as_uint(x);
    return __uint_as_float(__builtin_amdgcn_permlane16_swap(u, u, false, false)[1]);
}
__device__ __forceinline__ float lane_plus32(float x) {
    const unsigned u = __float_as_uint(x);
    return __uint_as_float(__builtin_amdgcn_permlane32_swap(u, u, false, false)[1]);
}

// Branch-free predicated stores through a raw buffer resource: a dropped lane gets an out-of-range offset and
// the hardware range check discards it. Inside sequential loops this keeps the VMEM stream straight-line, so
// the compiler's waitcnt for a prefetched load counts the stores issued after it (an `if (valid)` store would
// make it wait for every outstanding store instead). Element offsets must stay below 2^29 floats (host-checked).
typedef unsigned int mlg_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mlg_rsrc(const float* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st4_if(__amdgpu_buffer_rsrc_t rs, int64_t off, floatx4 v, bool keep) {
    const int byte = keep ? (int)(off * 4) : (int)0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(mlg_u32x4, v), rs, byte, 0, 0);
}

// 4x4 transpose across the four 16-lane rows of a wave (same lane within the row): on return x[g] in row p holds
// the input x[p] of row g. Two v_permlane16_swap + two v_permlane32_swap.
__device__ __forceinline__ void rows_transpose4(float& x0, float& x1, float& x2, float& x3) {
    const auto s01 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x0), __float_as_uint(x1), false, false);
    const auto s23 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x2), __float_as_uint(x3), false, false);
    const auto s02 = __builtin_amdgcn_permlane32_swap(s01[0], s23[0], false, false);
    const auto s13 = __builtin_amdgcn_permlane32_swap(s01[1], s23[1], false, false);
    x0 = __uint_as_float(s02[0]);
    x1 = __uint_as_float(s13[0]);
    x2 = __uint_as_float(s02[1]);
    x3 = __uint_as_float(s13[1]);
}
// Register-wise sum over the four 16-lane rows, transposed: row p receives (x[p]_row0 + x[p]_row1) +
// (x[p]_row2 + x[p]_row3). Three lane swaps and three adds.
__device__ __forceinline__ float rows_sum_transpose4(float x0, float x1, float x2, float x3) {
    const auto s01 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x0), __float_as_uint(x1), false, false);
    const auto s23 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x2), __float_as_uint(x3), false, false);
    const float a = __uint_as_float(s01[0]) + __uint_as_float(s01[1]);  // rows: x0 0+1, x1 0+1, x0 2+3, x1 2+3
    const float b = __uint_as_float(s23[0]) + __uint_as_float(s23[1]);  // same for x2, x3
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

// Inclusive prefix sum over groups of W lanes (W = 8 or 16, groups inside the 16-lane rows) on DPP row shifts --
// VALU moves -- instead of __shfl_up, which compiles to a chain of ds_bpermute LDS round trips. A lane whose shift
// source lies below its group's first lane adds 0.
template <int D>
__device__ __forceinline__ int dpp_row_shr(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x110 + D, 0xF, 0xF, false);
}
template <int W>
__device__ __forceinline__ int group_incl_scan(int c, int lane) {
    const int l = lane & (W - 1);
    int v = dpp_row_shr<1>(c);
    c += l >= 1 ? v : 0;
    v = dpp_row_shr<2>(c);
    c += l >= 2 ? v : 0;
    v = dpp_row_shr<4>(c);
    c += l >= 4 ? v : 0;
    if constexpr (W > 8) {
        v = dpp_row_shr<8>(c);
        c += l >= 8 ? v : 0;
    }
    return c;
}

// Raw buffer access with a per-lane byte offset vo and a wave-uniform (SGPR) byte offset so.
__device__ __forceinline__ floatx4 ld4_rs(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
    return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0));
}
__device__ __forceinline__ float ld1_rs(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, 0));
}
__device__ __forceinline__ void st1_rs(__amdgpu_buffer_rsrc_t rs, int vo, int so, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, vo, so, 0);
}
__device__ __forceinline__ void st4_rs(__amdgpu_buffer_rsrc_t rs, int vo, int so, floatx4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(mlg_u32x4, v), rs, vo, so, 0);
}

__device__ __forceinline__ floatx4 mfma_chunk(const floatx4 w, const floatx4 x, floatx4 acc) {
    acc = mfma4(w.x, x.x, acc);
    acc = mfma4(w.y, x.y, acc);
    acc = mfma4(w.z, x.z, acc);
    acc = mfma4(w.w, x.w, acc);
    return acc;
}

// ------------------------------------------------------------------------------------------------
// RNG (spec §3.7): rng(key, ctr) = splitmix64(key ^ splitmix64(ctr))
__device__ __forceinline__ uint64_t mlg_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t mlg_rng(uint64_t key, uint64_t ctr) { return mlg_splitmix64(key ^ mlg_splitmix64(ctr)); }
__device__ __forceinline__ uint64_t mlg_ctr(uint32_t episode, uint32_t t, uint32_t purpose, uint32_t idx) {
    return ((uint64_t)episode << 32) | ((uint64_t)(t & 0xFFFFu) << 16) | ((uint64_t)(purpose & 0xFu) << 12) |
           (uint64_t)(idx & 0xFFFu);
}
__device__ __forceinline__ float mlg_u01(uint64_t r) { return (float)(r >> 40) * (1.0f / 16777216.0f); }
__device__ __forceinline__ uint64_t mlg_env_key(uint64_t seed, int env) { return (seed << 32) + (uint64_t)env; }

enum { MLG_PURPOSE_SPAWN = 1, MLG_PURPOSE_EPS = 2, MLG_PURPOSE_RAND = 3 };

// ------------------------------------------------------------------------------------------------
// Env spec v1. Unit tables live in LDS, copied from the MlgEnvSpec kernel argument.
struct EnvTables {
    const int* team;   // [U]
    const int* role;   // [U]
    const int* melee;  // [U]
    const int* agent;  // [U] agent index + 1, 0 for scripted units
    int U, grid, episode_limit, stochastic;
};

__device__ __forceinline__ int role_maxhp(int r) { return r == 0 ? 64 : 32; }
__device__ __forceinline__ int role_power(int r) { return r == 0 ? 3 : (r == 1 ? 4 : 6); }
__device__ __forceinline__ int atk_range2(int melee) { return melee ? 2 : 9; }
__device__ __forceinline__ float inv_maxhp(int r) { return r == 0 ? (1.0f / 64.0f) : (1.0f / 32.0f); }

__device__ __forceinline__ int pow2_at_least(int g) {
    int p = 1;
    while (p < g) p <<= 1;
    return p;
}

__device__ __forceinline__ int env_dist2(const int* x, const int* y, int i, int j) {
    int dx = x[j] - x[i], dy = y[j] - y[i];
    return dx * dx + dy * dy;
}

// Availability of action a for unit i (spec §3.2).
__device__ __forceinline__ int env_avail_one(const EnvTables& T, const int* x, const int* y, const int* hp, int i, int a) {
    const int alive = hp[i] > 0;
    if (a == 0) return !alive;
    if (!alive) return 0;
    if (a == 1) return y[i] + 1 < T.grid;
    if (a == 2) return y[i] - 1 >= 0;
    if (a == 3) return x[i] + 1 < T.grid;
    if (a == 4) return x[i] - 1 >= 0;
    const int j = a - MLG_ACT_BASE;
    if (j < 0 || j >= T.U) return 0;
    if (hp[j] <= 0) return 0;
    if (env_dist2(x, y, i, j) > atk_range2(T.melee[i])) return 0;
    if (T.role[i] == 1) return j != i && T.team[j] == T.team[i] && hp[j] < role_maxhp(T.role[j]);
    return T.team[j] != T.team[i];
}

__device__ __forceinline__ int env_move_toward(const int* x, const int* y, int i, int j) {
    const int dx = x[j] - x[i], dy = y[j] - y[i];
    const int adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
    if (adx >= ady && dx != 0) return dx > 0 ? 3 : 4;
    if (dy != 0) return dy > 0 ? 1 : 2;
    return 0;
}

// Scripted "basic" AI (spec §3.3), decided on the pre-step state.
__device__ int env_ai_action(const EnvTables& T, const int* x, const int* y, const int* hp, int i) {
    if (hp[i] <= 0) return 0;
    int best = -1;
    for (int j = 0; j < T.U; ++j)
        if (env_avail_one(T, x, y, hp, i, MLG_ACT_BASE + j) && (best < 0 || hp[j] < hp[best])) best = j;
    if (best >= 0) return MLG_ACT_BASE + best;
    if (T.role[i] == 1) {
        int near = -1, nd = 0;
        for (int j = 0; j < T.U; ++j) {
            if (j == i || hp[j] <= 0 || T.team[j] != T.team[i]) continue;
            const int d = env_dist2(x, y, i, j);
            if (near < 0 || d < nd) { near = j; nd = d; }
        }
        if (near >= 0) return nd > 2 ? env_move_toward(x, y, i, near) : 0;
    }
    int near = -1, nd = 0;
    for (int j = 0; j < T.U; ++j) {
        if (hp[j] <= 0 || T.team[j] == T.team[i]) continue;
        const int d = env_dist2(x, y, i, j);
        if (near < 0 || d < nd) { near = j; nd = d; }
    }
    return near >= 0 ? env_move_toward(x, y, i, near) : 0;
}

__device__ __forceinline__ void env_spawn_xyh(const EnvTables& T, uint64_t key, uint32_t episode, int u, int team_first,
                                              int team_size, int& x, int& y, int& hp) {
    const int G = T.grid, tm = T.team[u];
    hp = role_maxhp(T.role[u]);
    if (T.stochastic) {
        const uint64_t r = mlg_rng(key, mlg_ctr(episode, 0, MLG_PURPOSE_SPAWN, (uint32_t)u));
        const int col = (int)(r % 4u);
        x = tm == 0 ? col : G - 1 - col;
        y = (int)((r >> 8) % (uint64_t)G);
    } else {
        const int k = u - team_first;
        x = tm == 0 ? 1 : G - 2;
        y = (k * G) / team_size + (G / team_size) / 2;
    }
}

__device__ __forceinline__ void env_spawn_unit(const EnvTables& T, uint64_t key, uint32_t episode, int u, int team_first,
                                               int team_size, int* x, int* y, int* hp) {
    env_spawn_xyh(T, key, episode, u, team_first, team_size, x[u], y[u], hp[u]);
}

// Obs features of unit j seen by unit i (spec §3.5): writes 8 floats.
__device__ __forceinline__ void env_obs_feat(const EnvTables& T, const int* x, const int* y, const int* hp, int i, int j,
                                             float inv_p, float* o) {
    if (hp[i] <= 0 || hp[j] <= 0 || env_dist2(x, y, i, j) > MLG_SIGHT2) {
#pragma unroll
        for (int f = 0; f < 8; ++f) o[f] = 0.0f;
        return;
    }
    o[0] = 1.0f;
    o[1] = (float)(x[j] - x[i]) * inv_p;
    o[2] = (float)(y[j] - y[i]) * inv_p;
    o[3] = (float)hp[j] * inv_maxhp(T.role[j]);
    o[4] = (float)env_avail_one(T, x, y, hp, i, MLG_ACT_BASE + j);
    o[5] = (float)(T.team[j] == T.team[i]);
    o[6] = (float)T.role[j] * 0.5f;
    o[7] = (float)T.melee[j];
}

__device__ __forceinline__ void env_state_feat(const EnvTables& T, const int* x, const int* y, const int* hp, int j,
                                               float inv_p, float* o) {
    o[0] = (float)(hp[j] > 0);
    o[1] = (float)x[j] * inv_p;
    o[2] = (float)y[j] * inv_p;
    o[3] = (float)hp[j] * inv_maxhp(T.role[j]);
    o[4] = (float)T.team[j];
    o[5] = (float)T.role[j] * 0.5f;
}

// Action actually executed by unit u: validated policy action or scripted AI action (spec §3.4).
__device__ __forceinline__ int env_exec_action(const EnvTables& T, const int* x, const int* y, const int* hp, int u,
                                               int64_t policy_action) {
    if (T.agent[u]) {
        const int a = (int)policy_action;
        return (a >= 0 && a < MLG_ACT_BASE + T.U && env_avail_one(T, x, y, hp, u, a)) ? a : 0;
    }
    return env_ai_action(T, x, y, hp, u);
}

// New hp of unit j given all executed actions (spec §3.4, simultaneous resolution). hp = pre-step.
__device__ __forceinline__ int env_resolve_hp(const EnvTables& T, const int* act, const int* hp, int j) {
    if (hp[j] <= 0) return hp[j];
    int dmg = 0, heal = 0;
    for (int i = 0; i < T.U; ++i) {
        if (hp[i] <= 0 || act[i] != MLG_ACT_BASE + j) continue;
        if (T.role[i] == 1) heal += role_power(1);
        else dmg += role_power(T.role[i]);
    }
    int v = hp[j] - dmg + heal;
    const int mx = role_maxhp(T.role[j]);
    return v < 0 ? 0 : (v > mx ? mx : v);
}

__device__ __forceinline__ void env_apply_move(int a, int* xu, int* yu) {
    if (a == 1) *yu += 1;
    else if (a == 2) *yu -= 1;
    else if (a == 3) *xu += 1;
    else if (a == 4) *xu -= 1;
}

// ------------------------------------------------------------------------------------------------
// argmax with torch.max semantics on CPU: NaN wins, ties -> lowest index.
__device__ __forceinline__ bool amax_better(float v, int i, float bv, int bi) {
    // branch-free form of: NaN beats any number (lowest index among NaNs), else larger value, ties -> lower index
    const bool vn = v != v, bn = bv != bv, lower = i < bi;
    const bool ord = (v > bv) | ((v == bv) & lower);
    return vn ? (!bn | lower) : (!bn & ord);
}
