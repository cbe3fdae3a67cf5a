// wgrad_device.h -- weight gradients as job lists, shared by the QMIX and REFIL learners:
// dW[M][K] = sum_rows delta[row][m] x[row][k], db[m] = sum_rows delta[row][m], split over 256-row chunks (one wave
// per (job, 16x16 tile, chunk), MFMA with the row index as K) and summed over chunks in a fixed order
// (deterministic). The reduce pass also emits per-block sums of squares for clip_grad_norm_.
#pragma once
#include <cstdlib>

#include "mlg_device.h"

namespace mlg {

constexpr int WCH = 256;  // rows per wgrad chunk

// ================================================================================================
// weight gradients: dW[M][K] = sum_rows delta[row][m] x[row][k], db[m] = sum_rows delta[row][m]
struct WJob {
    const float* delta;
    const float* x;
    float* dw;
    float* db;
    int64_t ldd, ldx;
    int M, K, rows, mt, nt, chunks;
    int task0;  // first task index
    int64_t slab0;
};
template <int MJ>
struct WJobsT {
    WJob j[MJ];
    int n;
};

template <int MJ>
__device__ __forceinline__ int find_job(const WJobsT<MJ>& J, int task) {
    int k = 0;
    while (k + 1 < J.n && J.j[k + 1].task0 <= task) ++k;
    return k;
}

// one wave per (job, m-tile, n-tile, row chunk); partial tile (+ bias partial when nt == 0) -> slab
template <int MJ>
__global__ void __launch_bounds__(256) wgrad_kernel(WJobsT<MJ> J, float* __restrict__ slab) {
    const int lane = threadIdx.x & 63;
    const int task = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (task >= J.j[J.n - 1].task0 + J.j[J.n - 1].mt * J.j[J.n - 1].nt * J.j[J.n - 1].chunks) return;
    const WJob jb = J.j[find_job(J, task)];
    const int local = task - jb.task0;
    const int ch = local % jb.chunks, tt = local / jb.chunks;
    const int mt = tt / jb.nt, nt = tt % jb.nt;
    const int col = lane & 15, g = lane >> 4;
    const int m = mt * 16 + col, k = nt * 16 + col;
    const int r0 = ch * WCH, r1 = min(jb.rows, r0 + WCH);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;
    const bool mv = m < jb.M, kv = k < jb.K;
    for (int rr = r0; rr < r1; rr += 4) {
        const int row = rr + g;
        const bool rv = row < r1;
        const float a = (mv && rv) ? jb.delta[(int64_t)row * jb.ldd + m] : 0.f;
        const float xv = (kv && rv) ? jb.x[(int64_t)row * jb.ldx + k] : 0.f;
        acc = mfma4(a, xv, acc);
        bsum += a;
    }
    float* out = slab + jb.slab0 + ((int64_t)tt * jb.chunks + ch) * 272;
    // D layout: reg q -> (m = mt*16 + 4g + q, k = nt*16 + col)
#pragma unroll
    for (int q = 0; q < 4; ++q) out[(4 * g + q) * 16 + col] = acc[q];
    bsum += __shfl_xor(bsum, 16);
    bsum += __shfl_xor(bsum, 32);
    if (g == 0) out[256 + col] = bsum;
}

// fixed-order sum over chunks -> dW, db
__device__ __forceinline__ float block_sum_1024(float v, float* red) {
    // deterministic sum over blockDim.x (a multiple of 64, <= 1024) threads, result in every thread: a butterfly
    // within each wave (lane 0's fixed association), then the waves' partials in wave order -- two barriers instead
    // of one per tree level
    const int tid = threadIdx.x, nw = (int)(blockDim.x >> 6);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    float r = 0.f;
    for (int i = 0; i < nw; ++i) r += red[i];
    __syncthreads();  // red reusable by the caller
    return r;
}

// slab partials -> dW / db; every block also emits the sum of squares of the gradients it wrote
template <int MJ>
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(WJobsT<MJ> J, const float* __restrict__ slab,
                                                           float* __restrict__ nrm_part) {
    __shared__ float red[256];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over (job, tile, 272)
    int64_t acc = 0;
    float sq = 0.f;
    for (int q = 0; q < J.n; ++q) {
        const WJob& jb = J.j[q];
        const int64_t n_el = (int64_t)jb.mt * jb.nt * 272;
        if (i >= acc && i < acc + n_el) {
            const int64_t loc = i - acc;
            const int tt = (int)(loc / 272), e = (int)(loc % 272);
            const int mt = tt / jb.nt, nt = tt % jb.nt;
            float s = 0.f;
            const float* base = slab + jb.slab0 + (int64_t)tt * jb.chunks * 272 + e;
            for (int ch = 0; ch < jb.chunks; ++ch) s += base[(int64_t)ch * 272];
            if (e < 256) {
                const int m = mt * 16 + e / 16, k = nt * 16 + e % 16;
                if (m < jb.M && k < jb.K) {
                    jb.dw[(int64_t)m * jb.K + k] = s;
                    sq = s * s;
                }
            } else if (nt == 0 && jb.db) {
                const int m = mt * 16 + (e - 256);
                if (m < jb.M) {
                    jb.db[m] = s;
                    sq = s * s;
                }
            }
            break;
        }
        acc += n_el;
    }
    const float bs = block_sum_1024(sq, red);
    if (threadIdx.x == 0) nrm_part[blockIdx.x] = bs;
}


inline WJob job(const float* delta, int64_t ldd, const float* x, int64_t ldx, float* dw, float* db, int M, int K, int rows) {
    WJob j;
    j.delta = delta;
    j.x = x;
    j.dw = dw;
    j.db = db;
    j.ldd = ldd;
    j.ldx = ldx;
    j.M = M;
    j.K = K;
    j.rows = rows;
    j.mt = (M + 15) / 16;
    j.nt = (K + 15) / 16;
    j.chunks = (rows + WCH - 1) / WCH;
    j.task0 = 0;
    j.slab0 = 0;
    return j;
}

// task / slab offsets of a job list; returns the slab floats (partials + per-block norm partials) and the task count
template <int MJ>
inline int64_t layout_jobs(WJobsT<MJ>& J, int* n_tasks, int64_t* n_red, int64_t* slab_part) {
    int tasks = 0;
    int64_t slab = 0, red = 0;
    for (int q = 0; q < J.n; ++q) {
        J.j[q].task0 = tasks;
        J.j[q].slab0 = slab;
        tasks += J.j[q].mt * J.j[q].nt * J.j[q].chunks;
        slab += (int64_t)J.j[q].mt * J.j[q].nt * J.j[q].chunks * 272;
        red += (int64_t)J.j[q].mt * J.j[q].nt * 272;
    }
    *n_tasks = tasks;
    *n_red = red;
    *slab_part = mlg_align4(slab);
    return mlg_align4(slab) + mlg_align4((red + 255) / 256);
}

}  // namespace mlg

// ================================================================================================
// Blocked variant: one wave per (job, 64 x 64 output block, 1024-row chunk); per 4-row step every lane loads 4 delta
// and 4 x values and issues 16 MFMAs (vs 2 loads per MFMA above); the 4 waves of a workgroup (4 chunks of one block)
// add their partials in LDS, partials [block][chunk group][64 * 64 + 64] summed over groups in a fixed order
// (deterministic).
namespace mlg {

constexpr int BCH = 1024;        // max rows per chunk
constexpr int BSLAB = 64 * 64 + 64;

struct BJob {
    const float* delta;
    const float* x;
    float* dw;
    float* db;
    int64_t ldd, ldx;
    int M, K, rows, mb, nb, chunks, ch_rows;
    int va, vb;  // delta / x rows readable as 16-byte vectors (ld % 4 == 0, 16-byte aligned base)
    int task0;
    int64_t slab0;
    // rows with an exactly zero delta skipped (REFIL learner: items past each sampled episode's live steps, whose
    // deltas the backward kernels write as zeros): 0 off; 1 item-major rows, item = (row / rpi) % I, (b, t) = (item / T,
    // item % T); 2 t-major rows, t = row / R, b = ((row % R) / NA) % B. Row r is live iff t < mlen[b]. Groups of 8
    // consecutive rows share one (b, t) (rpi, NA and R multiples of 8).
    int skip, rpi, I, T, R, NA, B;
    const float* mlen;
};
template <int MJ>
struct BJobsT {
    BJob j[MJ];
    int n;
};

inline BJob bjob(const float* delta, int64_t ldd, const float* x, int64_t ldx, float* dw, float* db, int M, int K,
                 int rows) {
    BJob j;
    j.delta = delta;
    j.x = x;
    j.dw = dw;
    j.db = db;
    j.ldd = ldd;
    j.ldx = ldx;
    j.M = M;
    j.K = K;
    j.rows = rows;
    j.mb = (M + 63) / 64;
    j.nb = (K + 63) / 64;
    // chunk length: up to BCH rows, fewer when the job is small so that it still spreads over >= ~256 waves
    static const int target = [] {  // waves per job (MLG_WGRAD_WAVES overrides, for tuning runs)
        const char* e = getenv("MLG_WGRAD_WAVES");
        const int v = e ? atoi(e) : 0;
        return v > 0 ? v : 256;
    }();
    int ch = rows / (target / (j.mb * j.nb) + 1);
    ch = ch < 64 ? 64 : (ch > BCH ? BCH : ch);
#if defined(MLG_WGRAD_F32)
    j.ch_rows = (ch + 3) & ~3;
#else
    j.ch_rows = (ch + 31) & ~31;  // whole 32-row MFMA steps
#endif
    j.va = (ldd % 4 == 0) && ((uintptr_t)delta % 16 == 0);
    j.vb = (ldx % 4 == 0) && ((uintptr_t)x % 16 == 0);
    j.chunks = (rows + j.ch_rows - 1) / j.ch_rows;
    j.task0 = 0;
    j.slab0 = 0;
    j.skip = 0;
    j.rpi = j.I = j.T = j.R = j.NA = j.B = 1;
    j.mlen = nullptr;
    return j;
}

// skip rows with zero deltas (see BJob::skip); item-major rows of rpi rows per item over I items of T steps
inline BJob bjob_items(BJob j, const float* mlen, int rpi, int I, int T) {
    j.skip = 1;
    j.mlen = mlen;
    j.rpi = rpi;
    j.I = I;
    j.T = T;
    return j;
}
// t-major rows: R rows per step, row r of a step belongs to episode (r / NA) % B
inline BJob bjob_steps(BJob j, const float* mlen, int R, int NA, int B) {
    j.skip = 2;
    j.mlen = mlen;
    j.R = R;
    j.NA = NA;
    j.B = B;
    return j;
}

__device__ __forceinline__ bool bjob_row_live(const BJob& jb, int row) {
    if (!jb.skip) return true;
    int b, t;
    if (jb.skip == 1) {
        const int item = (row / jb.rpi) % jb.I;
        b = item / jb.T;
        t = item % jb.T;
    } else {
        t = row / jb.R;
        b = ((row % jb.R) / jb.NA) % jb.B;
    }
    return t < (int)jb.mlen[b];
}

// row chunks are processed (and their partials stored) in groups of 4, one workgroup per group and output block
__host__ __device__ __forceinline__ int bjob_groups(const BJob& jb) { return (jb.chunks + 3) >> 2; }
// workgroups of a job: jobs with several output blocks take the groups in stripes of 8 (see wgrad_block_body), the
// last stripe padded with idle workgroups
__host__ __device__ __forceinline__ int bjob_stripe(const BJob& jb) { return jb.mb * jb.nb > 1 ? 8 : 1; }
__host__ __device__ __forceinline__ int bjob_wgs(const BJob& jb) {
    const int st = bjob_stripe(jb);
    return jb.mb * jb.nb * ((bjob_groups(jb) + st - 1) / st * st);
}

template <int MJ>
__device__ __forceinline__ int find_bjob(const BJobsT<MJ>& J, int task) {
    int k = 0;
    while (k + 1 < J.n && J.j[k + 1].task0 <= task) ++k;
    return k;
}

#if !defined(MLG_WGRAD_F32)
// the 8 rows rr + 8g .. rr + 8g + 7 of a lane: delta columns m0 .. m0 + 3 into a, x columns k0 .. k0 + 3 into b
// (zeros for a dead group / rows past rend / columns past M, K)
__device__ __forceinline__ void wgrad_load_step(const BJob& jb, int rr, int g, bool glive, int rend, int m0, int k0,
                                                bool va, bool vb, float (&a)[8][4], float (&b)[8][4]) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const int row = rr + 8 * g + t;
        const bool rv = glive && row < rend;
        const float* dr = jb.delta + (int64_t)row * jb.ldd + m0;
        const float* xr = jb.x + (int64_t)row * jb.ldx + k0;
        if (rv && va) {
            const floatx4 v = ld4(dr);
#pragma unroll
            for (int i = 0; i < 4; ++i) a[t][i] = v[i];
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) a[t][i] = (rv && m0 + i < jb.M) ? dr[i] : 0.f;
        }
        if (rv && vb) {
            const floatx4 v = ld4(xr);
#pragma unroll
            for (int i = 0; i < 4; ++i) b[t][i] = v[i];
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) b[t][i] = (rv && k0 + i < jb.K) ? xr[i] : 0.f;
        }
    }
}

// one 32-row step's products: tile i's A operand is element i of the 8 delta vectors, tile j's B operand element j
// of the 8 x vectors; x tiles split one at a time (12 VGPRs live instead of 48); every accumulator sees the same
// product sequence as with all four split up front
__device__ __forceinline__ void wgrad_mfma_step(const float (&a)[8][4], const float (&b)[8][4], floatx4 (&acc)[4][4],
                                                float (&bsum)[4]) {
    Split3 as[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        as[i] = split3(floatx4{a[0][i], a[1][i], a[2][i], a[3][i]}, floatx4{a[4][i], a[5][i], a[6][i], a[7][i]});
#pragma unroll
        for (int t = 0; t < 8; ++t) bsum[i] += a[t][i];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const Split3 bs = split3(floatx4{b[0][j], b[1][j], b[2][j], b[3][j]}, floatx4{b[4][j], b[5][j], b[6][j], b[7][j]});
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][j] = mfma_x6(as[i], bs, acc[i][j]);
    }
}
#endif

// the work of workgroup `bid` (4 waves = 4 consecutive tasks) of a wgrad launch; a __device__ function so that
// a learner can run it as extra workgroups of another launch (learner.hip bwd4_wgrad_kernel). 256 threads.
template <int MJ, bool GLDS = false>
__device__ __forceinline__ void wgrad_block_body(const BJobsT<MJ>& J, float* __restrict__ slab, int bid) {
    // partials of the 4 waves summed pairwise in LDS, (c0 + c2) + (c1 + c3), before the one slab store per workgroup
    // (two 16 KB slots: with the reverse recurrence's LDS, bwd4_wgrad_kernel still fits two workgroups per CU). GLDS:
    // 16 KB of row staging per wave, the slots in waves 2 and 3's staging (their loops are over when they fill them)
    __shared__ __attribute__((aligned(16))) floatx4 lbuf[GLDS ? 4 : 2][16][64];
    floatx4(*wred)[16][64] = GLDS ? lbuf + 2 : lbuf;
    __shared__ float wbred[2][4][16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int task = bid * 4 + w;
    const BJob& last = J.j[J.n - 1];
    // job task counts are multiples of 4: the test (and the job) is the same for the whole workgroup
    if (bid * 4 >= last.task0 + bjob_wgs(last) * 4) return;
    const BJob jb = J.j[find_bjob(J, task)];
    const int wg = (task - jb.task0) >> 2;
    // the 4 waves of a workgroup take the row chunks 4 cg .. 4 cg + 3 of one 64 x 64 output block and add their
    // partials in LDS, so the slab holds one partial per chunk group. Jobs with several output blocks (M = 192:
    // in_trans, W_ih, W_hh; K > 64) take the groups in stripes of 8: workgroup wg of a stripe has group
    // stripe * 8 + wg % 8 and block wg / 8, so the blocks of one group are 8 workgroups apart - dispatched at about
    // the same time to the same XCD (round-robin over the 8 XCDs), where the first to read a row chunk brings it into
    // that XCD's L2 for the others
    const int nblk = jb.mb * jb.nb, st = bjob_stripe(jb);
    const int sl = wg / (st * nblk), sr = wg % (st * nblk);
    const int cg = sl * st + sr % st, blk = sr / st;
    if (cg >= bjob_groups(jb)) return;  // the last stripe's padding (whole workgroup)
    const int ch = 4 * cg + w;
    const bool act = ch < jb.chunks;  // the last group's spare waves add zeros
    const int mbi = blk / jb.nb, nbi = blk % jb.nb;
    const int col = lane & 15, g = lane >> 4;
    const int r0 = ch * jb.ch_rows, r1 = act ? min(jb.rows, r0 + jb.ch_rows) : r0;
    floatx4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};
    // lane col reads the 4 consecutive delta columns m0 .. m0 + 3 and x columns k0 .. k0 + 3 of its row (one 16-byte
    // load each when the row layout allows it): MFMA tile i holds m = m0 + i, tile j holds k = k0 + j. The row (K)
    // order of every product is unchanged; only the block's output positions are permuted (undone at the store).
    const int m0 = mbi * 64 + 4 * col, k0 = nbi * 64 + 4 * col;
    const bool va = jb.va && m0 + 3 < jb.ldd, vb = jb.vb && k0 + 3 < jb.ldx;
#if !defined(MLG_WGRAD_F32)
    // 32-row steps on the bf16 matrix cores as split-bf16 fp32 emulation (six partial products, fp32 accumulation,
    // mlg_device.h mfma_x6): lane (col, g) loads rows rr + 8g .. rr + 8g + 7; K slot t of its operands = row
    // rr + 8g + t, so tile i's A operand is element i of the 8 delta vectors and tile j's B operand element j of
    // the 8 x vectors. Same D layout (and output permutation) as the f32 form below.
    // jobs that skip dead rows deal their 32-row steps to the chunks round-robin (chunk ch takes steps ch, ch +
    // chunks, ...): the live rows (a prefix of every episode) then spread evenly over the job's waves instead of
    // leaving whole chunks with all the work; other jobs keep contiguous chunks
    const bool strided = jb.skip != 0;
    const int s0 = strided ? ch : r0 >> 5, s1 = !act ? s0 : strided ? (jb.rows + 31) >> 5 : (r1 + 31) >> 5;
    const int ds = strided ? jb.chunks : 1, rend = strided ? jb.rows : r1;
    // rows with zero deltas add exactly zero: a lane's 8-row group of them loads nothing (zeros), a step with no live
    // group is skipped. The wave's steps are indexed i = 0 .. nst - 1 (step s0 + i ds); their liveness is evaluated
    // 64 steps at a time, lane l taking step index 64 win + l for the 4 row groups (four ballots), so the loop itself
    // does no integer division. With <= 64 episodes the episode lengths sit in a register (episode e in lane e).
    const int nst = act ? (s1 - s0 + ds - 1) / ds : 0;
    const int nep = jb.skip == 1 ? jb.I / jb.T : jb.B;
    const bool mreg = jb.skip && nep <= 64;
    const float mlv = (mreg && lane < nep) ? jb.mlen[lane] : 0.f;
    int win = -1;
    uint64_t any = 0, mg = 0;  // steps of the window with a live group; this lane's group's live steps
    auto group_live = [&](int row) -> bool {
        bool gv = row < rend;
        if (jb.skip) {
            int eb, et;
            if (jb.skip == 1) {
                const int item = (row / jb.rpi) % jb.I;
                eb = item / jb.T;
                et = item % jb.T;
            } else {
                et = row / jb.R;
                eb = ((row % jb.R) / jb.NA) % jb.B;
            }
            const float ml = mreg ? __shfl(mlv, eb & 63) : (gv ? jb.mlen[eb] : 0.f);
            gv = gv && et < (int)ml;
        }
        return gv;
    };
    auto next_live = [&](int i) -> int {  // first step index >= i with a live group (nst: none)
        while (i < nst) {
            if ((i >> 6) != win) {
                win = i >> 6;
                const int li = (win << 6) + lane;
                const int rl = (s0 + li * ds) << 5;
                const bool inr = li < nst;
                // group_live first: its lane shuffle runs with every lane active
                const uint64_t b0 = __ballot(group_live(rl) && inr), b1 = __ballot(group_live(rl + 8) && inr),
                               b2 = __ballot(group_live(rl + 16) && inr), b3 = __ballot(group_live(rl + 24) && inr);
                any = b0 | b1 | b2 | b3;
                mg = g == 0 ? b0 : g == 1 ? b1 : g == 2 ? b2 : b3;
            }
            const uint64_t rem = any & (~0ull << (i & 63));
            if (rem) return (win << 6) + __builtin_ctzll(rem);
            i = (win + 1) << 6;
        }
        return nst;
    };
    auto live_of = [&](int i) -> bool { return (mg >> (i & 63)) & 1; };  // i in the current window
    int i = next_live(0);
    bool gl = i < nst && live_of(i);
    if constexpr (GLDS) {
        // one step ahead through LDS: the next live step's 16 row loads go global -> LDS (global_load_lds, 16 bytes
        // per lane, this wave's 16 KB of `lbuf`) while this step's products run from VGPRs (a register copy of the
        // next step does not fit in 256 VGPRs). Lanes whose rows are dead or past the end load row 0 and are zeroed
        // after the read (columns past M / K are loaded as in the register path: they only reach discarded output
        // rows / columns).
        if (__all(va && vb)) {
            floatx4(*stg)[64] = lbuf[w];
            auto issue = [&](int ii, bool gv) {
                const int rr = (s0 + ii * ds) << 5;
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const int row = rr + 8 * g + t;
                    const int64_t rs = (gv && row < rend) ? row : 0;
                    __builtin_amdgcn_global_load_lds((const void*)(jb.delta + rs * jb.ldd + m0),
                                                     (__attribute__((address_space(3))) void*)&stg[t][0], 16, 0, 0);
                    __builtin_amdgcn_global_load_lds((const void*)(jb.x + rs * jb.ldx + k0),
                                                     (__attribute__((address_space(3))) void*)&stg[8 + t][0], 16, 0, 0);
                }
            };
            if (i < nst) issue(i, gl);
            while (i < nst) {
                const int in = next_live(i + 1);
                const bool gn = in < nst && live_of(in);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const int rr = (s0 + i * ds) << 5;
                float a[8][4], b[8][4];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const bool rv = gl && rr + 8 * g + t < rend;
                    const floatx4 va4 = stg[t][lane], vb4 = stg[8 + t][lane];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        a[t][q] = rv ? va4[q] : 0.f;
                        b[t][q] = rv ? vb4[q] : 0.f;
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the reads are done before the buffer refills
                if (in < nst) issue(in, gn);
                wgrad_mfma_step(a, b, acc, bsum);
                i = in;
                gl = gn;
            }
        }
    }
    while (i < nst) {
        float a[8][4], b[8][4];
        wgrad_load_step(jb, (s0 + i * ds) << 5, g, gl, rend, m0, k0, va, vb, a, b);
        wgrad_mfma_step(a, b, acc, bsum);
        i = next_live(i + 1);
        gl = i < nst && live_of(i);
    }
#else
    // two 4-row steps per iteration: both steps' loads are issued before the first step's MFMAs (same
    // accumulation order as one step per iteration)
    for (int rr = r0; rr < r1; rr += 8) {
        float a[2][4], b[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = rr + 4 * h + g;
            const bool rv = row < r1;
            const float* dr = jb.delta + (int64_t)row * jb.ldd + m0;
            const float* xr = jb.x + (int64_t)row * jb.ldx + k0;
            if (rv && va) {
                const floatx4 v = ld4(dr);
#pragma unroll
                for (int i = 0; i < 4; ++i) a[h][i] = v[i];
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) a[h][i] = (rv && m0 + i < jb.M) ? dr[i] : 0.f;
            }
            if (rv && vb) {
                const floatx4 v = ld4(xr);
#pragma unroll
                for (int i = 0; i < 4; ++i) b[h][i] = v[i];
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) b[h][i] = (rv && k0 + i < jb.K) ? xr[i] : 0.f;
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h == 1 && rr + 4 >= r1) break;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                bsum[i] += a[h][i];
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = mfma4(a[h][i], b[h][j], acc[i][j]);
            }
        }
    }
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        bsum[i] += __shfl_xor(bsum[i], 16);
        bsum[i] += __shfl_xor(bsum[i], 32);
    }
    auto put = [&](int v) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) wred[v][4 * i + j][lane] = acc[i][j];
        if (g == 0)
#pragma unroll
            for (int i = 0; i < 4; ++i) wbred[v][i][col] = bsum[i];
    };
    auto add = [&](int v) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] += wred[v][4 * i + j][lane];
            bsum[i] += wbred[v][i][col];
        }
    };
    if (w >= 2) put(w - 2);
    __syncthreads();
    if (w < 2) add(w);
    if (w == 1) put(1);  // slot 1 was read by this wave only
    __syncthreads();
    if (w != 0) return;
    add(1);
    float* out = slab + jb.slab0 + ((int64_t)blk * bjob_groups(jb) + cg) * BSLAB;
    // D layout: acc[i][j] reg q -> MFMA row 4g + q, i.e. the A values of lane col' = 4g + q (block row
    // m = 4 col' + i), and MFMA column col (block column k = 4 col + j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<floatx4*>(out + (4 * (4 * g + q) + i) * 64 + 4 * col) =
                floatx4{acc[i][0][q], acc[i][1][q], acc[i][2][q], acc[i][3][q]};
    if (g == 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) out[4096 + 4 * col + i] = bsum[i];
}

// fixed-order sum over chunk groups -> dW / db (bias from the nbi == 0 blocks); per-block sums of squares -> nrm_part
template <int MJ>
__global__ void __launch_bounds__(256, 2) wgrad_block_kernel(BJobsT<MJ> J, float* __restrict__ slab) {
#if defined(MLG_WGRAD_NOGLDS)
    wgrad_block_body<MJ, false>(J, slab, (int)blockIdx.x);
#else
    wgrad_block_body<MJ, true>(J, slab, (int)blockIdx.x);
#endif
}

template <int MJ>
__global__ void __launch_bounds__(256) wgrad_block_reduce_kernel(BJobsT<MJ> J, const float* __restrict__ slab,
                                                                 float* __restrict__ nrm_part) {
    __shared__ float red[256];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t acc = 0;
    float sq = 0.f;
    for (int q = 0; q < J.n; ++q) {
        const BJob& jb = J.j[q];
        const int64_t n_el = (int64_t)jb.mb * jb.nb * BSLAB;
        if (i >= acc && i < acc + n_el) {
            const int64_t loc = i - acc;
            const int blk = (int)(loc / BSLAB), e = (int)(loc % BSLAB);
            const int mbi = blk / jb.nb, nbi = blk % jb.nb;
            float s = 0.f;
            const int ng = bjob_groups(jb);
            const float* base = slab + jb.slab0 + (int64_t)blk * ng * BSLAB + e;
            int ch = 0;
#ifndef MLG_WRED_DEPTH
#define MLG_WRED_DEPTH 64
#endif
            // MLG_WRED_DEPTH loads in flight (the slab partials were just written by other CUs: each round trip is an
            // L2 / MALL miss), summed in group order
            for (; ch + MLG_WRED_DEPTH <= ng; ch += MLG_WRED_DEPTH) {
                float v[MLG_WRED_DEPTH];
#pragma unroll
                for (int u = 0; u < MLG_WRED_DEPTH; ++u) v[u] = base[(int64_t)(ch + u) * BSLAB];
#pragma unroll
                for (int u = 0; u < MLG_WRED_DEPTH; ++u) s += v[u];
            }
            for (; ch + 8 <= ng; ch += 8) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = base[(int64_t)(ch + u) * BSLAB];
#pragma unroll
                for (int u = 0; u < 8; ++u) s += v[u];
            }
            for (; ch < ng; ++ch) s += base[(int64_t)ch * BSLAB];
            if (e < 4096) {
                const int m = mbi * 64 + e / 64, k = nbi * 64 + e % 64;
                if (m < jb.M && k < jb.K) {
                    jb.dw[(int64_t)m * jb.K + k] = s;
                    sq = s * s;
                }
            } else if (nbi == 0 && jb.db) {
                const int m = mbi * 64 + (e - 4096);
                if (m < jb.M) {
                    jb.db[m] = s;
                    sq = s * s;
                }
            }
            break;
        }
        acc += n_el;
    }
    const float bs = block_sum_1024(sq, red);
    if (threadIdx.x == 0) nrm_part[blockIdx.x] = bs;
}

template <int MJ>
inline int64_t layout_bjobs(BJobsT<MJ>& J, int* n_tasks, int64_t* n_red, int64_t* slab_part) {
    int tasks = 0;
    int64_t slab = 0, red = 0;
    for (int q = 0; q < J.n; ++q) {
        J.j[q].task0 = tasks;
        J.j[q].slab0 = slab;
        tasks += bjob_wgs(J.j[q]) * 4;
        slab += (int64_t)J.j[q].mb * J.j[q].nb * bjob_groups(J.j[q]) * BSLAB;
        red += (int64_t)J.j[q].mb * J.j[q].nb * BSLAB;
    }
    *n_tasks = tasks;
    *n_red = red;
    *slab_part = mlg_align4(slab);
    // norm partials: one per reduce block, + 4 for a table reduced as two views (bjob_view: one more block at most)
    return mlg_align4(slab) + mlg_align4((red + 255) / 256) + 4;
}

// jobs [q0, q1) of a laid-out table as a table of their own (tasks renumbered from 0, slab positions kept): the
// wgrad and reduce launches of a view compute exactly the view's dW / db (same chunks, same order), so a table can
// run as two views on two streams; the view's norm partials go to their own range of the partial array
template <int MJ>
inline BJobsT<MJ> bjob_view(const BJobsT<MJ>& J, int q0, int q1, int* n_tasks, int64_t* n_red) {
    BJobsT<MJ> V;
    V.n = 0;
    int tasks = 0;
    int64_t red = 0;
    for (int q = q0; q < q1; ++q) {
        V.j[V.n] = J.j[q];
        V.j[V.n].task0 = tasks;
        tasks += bjob_wgs(J.j[q]) * 4;
        red += (int64_t)J.j[q].mb * J.j[q].nb * BSLAB;
        ++V.n;
    }
    *n_tasks = tasks;
    *n_red = red;
    return V;
}

}  // namespace mlg
