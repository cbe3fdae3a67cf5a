// rollout.hip -- the fused ParallelStepper.run kernel and the standalone env kernels.
//
// One launch = one ParallelStepper.run (src/steppers/parallel_stepper.py:106-216) over all B envs:
// reset (:82-104), then per timestep t the batched agent step (BasicMAC.select_actions ->
// DRQN forward -> epsilon-greedy, basic_controller.py:29-36, action_selectors.py:44-62) and the
// batched env step that replaces B EnvWorker processes (env_worker_process.py:32-53).
//
// Envs are independent, so a workgroup owns RE = 16 envs for the whole episode: GRU hidden state
// stays in VGPRs, env state in LDS, nothing crosses workgroups and there is no grid barrier.
// Workgroup = W waves (W = min(ceil(16*N/16), 8)); wave w owns the 16-row agent tiles w, w+W, ...
// (row = env * N + agent).  Per timestep:
//   agent phase (MFMA cell per tile; masked argmax/eps over 64 lanes with 2 shuffles) ->
//   barrier -> env phase (one thread per (env, unit): AI actions, simultaneous resolution,
//   per-env reductions) -> obs/state/avail of t+1 straight into the EpisodeBatch in HBM.
// Bookkeeping is the reference's intended one: an env that terminates while
// stepping at t still receives (and records) an action at t+1, then stops.
#include "agent_device.h"
#include "mlg_host.h"

#ifdef MLG_STAMPS
// Diagnostic build only (-DMLG_STAMPS, libmaleague_stamps.so): per-wave cycle shares of the rollout phases.
__device__ unsigned long long* g_mlg_stamps = nullptr;
#define MLG_STAMP(k)                                             \
    do {                                                         \
        const unsigned long long _now = __builtin_amdgcn_s_memtime(); \
        st_acc[k] += _now - st_last;                             \
        st_last = _now;                                          \
    } while (0)
#else
#define MLG_STAMP(k) \
    do {             \
    } while (0)
#endif

namespace {

constexpr int RE = 16;  // envs per workgroup

struct SpecShared {
    int team[MLG_MAXU], role[MLG_MAXU], melee[MLG_MAXU], agent[MLG_MAXU];
    int team_first[2], team_size[2];
};

__device__ void load_spec_tables(const MlgEnvSpec& spec, SpecShared& s) {
    const int tid = threadIdx.x;
    for (int u = tid; u < MLG_MAXU; u += blockDim.x) {
        const bool in = u < spec.U;
        s.team[u] = in ? spec.team[u] : 0;
        s.role[u] = in ? spec.role[u] : 0;
        s.melee[u] = in ? spec.melee[u] : 0;
        s.agent[u] = 0;
    }
    __syncthreads();
    for (int a = tid; a < spec.n_agents; a += blockDim.x) s.agent[spec.agent_unit[a]] = a + 1;
    if (tid == 0) {
        for (int tm = 0; tm < 2; ++tm) {
            s.team_first[tm] = -1;
            s.team_size[tm] = 0;
        }
        for (int u = 0; u < spec.U; ++u) {
            const int tm = spec.team[u];
            if (s.team_first[tm] < 0) s.team_first[tm] = u;
            s.team_size[tm]++;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ EnvTables make_tables(const MlgEnvSpec& spec, const SpecShared& s) {
    EnvTables T;
    T.team = s.team;
    T.role = s.role;
    T.melee = s.melee;
    T.agent = s.agent;
    T.U = spec.U;
    T.grid = spec.grid;
    T.episode_limit = spec.episode_limit;
    T.stochastic = spec.stochastic;
    return T;
}

// Writes obs/state/avail of env (x,y,hp) for batch slot (b, t); called cooperatively:
// item index i in [0, items) distributed over the threads of the block by the caller.
__device__ __forceinline__ void write_obs_item(const EnvTables& T, const MlgEnvSpec& spec, const int* x, const int* y,
                                               const int* hp, float* obs_bt, int a, int j, float inv_p) {
    float o[8];
    env_obs_feat(T, x, y, hp, spec.agent_unit[a], j, inv_p, o);
    float* dst = obs_bt + ((int64_t)a * T.U + j) * 8;
    *reinterpret_cast<floatx4*>(dst) = floatx4{o[0], o[1], o[2], o[3]};
    *reinterpret_cast<floatx4*>(dst + 4) = floatx4{o[4], o[5], o[6], o[7]};
}

// Zero every key of slots [t0, t1) of the envs of this workgroup that are done and did not step
// (status 2, or stepped == 0 with status 2 after the final action): the full-write (ring) mode's
// replacement for zero-initialising the EpisodeBatch.
__device__ void zero_slots(const MlgBatch& bt, const int* s_slot, const int* s_status, const int* s_stepped, int e0,
                           int B, int t0, int t1, int N, int A, int S, int DO) {
    const int T1 = bt.T1;
    const int per = S + N * DO + 2 * N * A + 2 * N + 3;  // words per slot (actions/filled are 2 words)
    const int total = RE * (t1 - t0) * per;
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
        const int e = i / ((t1 - t0) * per), rem = i % ((t1 - t0) * per);
        const int t = t0 + rem / per;
        int k = rem % per;
        if (e0 + e >= B || s_status[e] != 2 || s_stepped[e]) continue;
        const int64_t sl = (int64_t)s_slot[e] * T1 + t;
        if (k < S) { bt.state[sl * S + k] = 0.f; continue; }
        k -= S;
        if (k < N * DO) { bt.obs[sl * N * DO + k] = 0.f; continue; }
        k -= N * DO;
        if (k < N * A) { bt.avail[sl * N * A + k] = 0; continue; }
        k -= N * A;
        if (k < N * A) { bt.actions_onehot[sl * N * A + k] = 0.f; continue; }
        k -= N * A;
        if (k < N) { bt.actions[sl * N + k] = 0; continue; }
        k -= N;
        if (k < N) continue;  // (second word of the int64 actions, covered above)
        k -= N;
        if (k == 0) bt.reward[sl] = 0.f;
        else if (k == 1) bt.terminated[sl] = 0;
        else bt.filled[sl] = 0;
    }
}

// Dynamic-LDS carve of the rollout workgroup (4-byte words; every region 16-byte aligned).
struct RolloutLds {
    int64_t wts, spec, x, y, hp, nhp, act, pact, prev, status, stepped, len, episode, ret, slot, any, total;
    LdsWeights lw;
    int weights_in_lds;
};

__host__ __device__ inline RolloutLds make_rollout_lds(const AgentLayout& L, int U, int n_agents, bool weights_in_lds) {
    RolloutLds r;
    r.lw = make_lds_weights(L);
    r.weights_in_lds = weights_in_lds;
    int64_t o = 0;
    auto take = [&](int64_t n) { int64_t v = o; o += mlg_align4(n); return v; };
    r.wts = take(weights_in_lds ? r.lw.total : 0);
    r.spec = take((int64_t)(sizeof(SpecShared) / 4));
    const int64_t eu = (int64_t)RE * U;
    r.x = take(eu);
    r.y = take(eu);
    r.hp = take(eu);
    r.nhp = take(eu);
    r.act = take(eu);
    r.pact = take((int64_t)RE * n_agents);
    r.prev = take((int64_t)RE * n_agents);
    r.status = take(RE);
    r.stepped = take(RE);
    r.len = take(RE);
    r.episode = take(RE);
    r.ret = take(RE);
    r.slot = take(RE);
    r.any = take(1);
    r.total = o;
    return r;
}

template <int H, int TPW, bool WLDS>
__global__ void __launch_bounds__(512) rollout_kernel(MlgEnvSpec spec, MlgEnvState st, AgentLayout L,
                                                     const float* __restrict__ P, MlgBatch bt, MlgRunInfo info,
                                                     float eps, int test_mode, RolloutLds lay) {
    constexpr int HC = H / 16;
    extern __shared__ __attribute__((aligned(16))) int smem[];
    SpecShared& SS = *reinterpret_cast<SpecShared*>(smem + lay.spec);
    const int U = spec.U, N = spec.n_agents, A = spec.n_actions, S = 6 * U, DO = 8 * U;
    int* s_x = smem + lay.x;
    int* s_y = smem + lay.y;
    int* s_hp = smem + lay.hp;
    int* s_nhp = smem + lay.nhp;
    int* s_act = smem + lay.act;
    int* s_pact = smem + lay.pact;
    int* s_prev = smem + lay.prev;
    int* s_status = smem + lay.status;
    int* s_stepped = smem + lay.stepped;
    int* s_len = smem + lay.len;
    uint32_t* s_episode = reinterpret_cast<uint32_t*>(smem + lay.episode);
    float* s_ret = reinterpret_cast<float*>(smem + lay.ret);
    int* s_slot = smem + lay.slot;  // batch slot of env e (ring mode: the replay-buffer slot)
    int& s_any = smem[lay.any];

    const int tid = threadIdx.x, nthr = blockDim.x;
    const int lane = tid & 63, wave = tid >> 6, W = nthr >> 6;
    const int e0 = blockIdx.x * RE;
    const int B = bt.B, T1 = bt.T1;
    load_spec_tables(spec, SS);
    if (WLDS) load_weights_to_lds(P, L, lay.lw, reinterpret_cast<float*>(smem + lay.wts));
    const EnvTables T = make_tables(spec, SS);
    const float inv_p = 1.0f / (float)pow2_at_least(spec.grid);

    // ---- reset (parallel_stepper.py:82-104; env_worker_process.py:54-60) ----
    for (int e = tid; e < RE; e += nthr) {
        const int b = e0 + e;
        s_len[e] = 0;
        s_ret[e] = 0.f;
        s_stepped[e] = 0;
        if (b < B) {
            const uint32_t ep = st.episode[b];
            st.episode[b] = ep + 1;
            s_episode[e] = ep;
            s_status[e] = 0;
            const int sl = bt.ring_size > 0 ? (bt.ring_slot0 + b) % bt.ring_size : b;
            s_slot[e] = sl;
            bt.filled[(int64_t)sl * T1] = 1;
        } else {
            s_status[e] = 2;
        }
    }
    __syncthreads();
    for (int i = tid; i < RE * U; i += nthr) {
        const int e = i / U, u = i % U;
        if (s_status[e] == 2) continue;
        const int tm = SS.team[u];
        env_spawn_unit(T, mlg_env_key(spec.seed, e0 + e), s_episode[e], u, SS.team_first[tm], SS.team_size[tm],
                       s_x + e * U, s_y + e * U, s_hp + e * U);
    }
    __syncthreads();
    // observation at t = 0
    for (int i = tid; i < RE * N * U; i += nthr) {
        const int e = i / (N * U), r = i % (N * U);
        if (s_status[e] == 2) continue;
        write_obs_item(T, spec, s_x + e * U, s_y + e * U, s_hp + e * U, bt.obs + (int64_t)s_slot[e] * T1 * N * DO, r / U,
                       r % U, inv_p);
    }
    for (int i = tid; i < RE * U; i += nthr) {
        const int e = i / U, j = i % U;
        if (s_status[e] == 2) continue;
        float o[6];
        env_state_feat(T, s_x + e * U, s_y + e * U, s_hp + e * U, j, inv_p, o);
        float* dst = bt.state + (int64_t)s_slot[e] * T1 * S + j * 6;
#pragma unroll
        for (int f = 0; f < 6; ++f) dst[f] = o[f];
    }
    for (int i = tid; i < RE * N * A; i += nthr) {
        const int e = i / (N * A), r = i % (N * A);
        if (s_status[e] == 2) continue;
        bt.avail[(int64_t)s_slot[e] * T1 * N * A + r] =
            env_avail_one(T, s_x + e * U, s_y + e * U, s_hp + e * U, spec.agent_unit[r / A], r % A);
    }
    __syncthreads();

    floatx4 h[TPW][HC];
#pragma unroll
    for (int ti = 0; ti < TPW; ++ti)
#pragma unroll
        for (int c = 0; c < HC; ++c) h[ti][c] = floatx4{0.f, 0.f, 0.f, 0.f};
#ifdef MLG_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
    const unsigned long long st_begin = st_last;
#endif

    const int n_tiles = (RE * N + 15) / 16;
    const int col = lane & 15, g = lane >> 4;
    const int n_at = L.Ap / 16;
    int last_t = 0;

    for (int t = 0; t < T1; ++t) {
        // ================= agent phase: rows of envs with status 0 (running) or 1 (final action) ======
#pragma unroll
        for (int ti = 0; ti < TPW; ++ti) {
            const int tile = wave + ti * W;
            if (tile >= n_tiles) continue;
            const int row = tile * 16 + col;
            const int e = row / N, n = row % N;
            const bool valid = row < RE * N && s_status[e] < 2;
            if (!__any(valid)) continue;  // wave-uniform skip of finished tiles
            // Opaque zero offset per tile: stops LICM/CSE from keeping t- and tile-invariant weight loads
            // live across the episode loop in (spilled) registers.
            int zero = 0;
            asm volatile("" : "+s"(zero));
            const WView Wv = WLDS ? lds_view(reinterpret_cast<const float*>(smem + lay.wts) + zero, lay.lw, L)
                                  : global_view(P + zero, L);
            const int64_t b = e0 + e;
            const int64_t bt_off = valid ? ((int64_t)s_slot[e] * T1 + t) * N + n : 0;
            RowIn in;
            in.x = valid ? bt.obs + bt_off * DO : nullptr;
            in.onehot = nullptr;
            in.prev_action = (valid && t > 0) ? s_prev[e * N + n] : -1;
            in.agent = valid ? n : 0;
            agent_cell_hidden<H>(Wv, L, in, h[ti], lane);
            const int32_t* av = valid ? bt.avail + bt_off * A : nullptr;
            ArgmaxState as{-INFINITY, 1 << 30};
            for (int at = 0; at < n_at; ++at) {
                const floatx4 q = agent_q_tile<H>(Wv, h[ti], at, lane);
                argmax_accumulate(as, q, av, at, A, lane);
            }
            int act = argmax_reduce(as);
            if (valid && g == 0) {
                if (!test_mode && eps > 0.f) {
                    const uint64_t key = mlg_env_key(spec.seed, (int)b);
                    const uint64_t r1 = mlg_rng(key, mlg_ctr(s_episode[e], (uint32_t)t, MLG_PURPOSE_EPS, (uint32_t)n));
                    if (mlg_u01(r1) < eps) {
                        const uint64_t r2 = mlg_rng(key, mlg_ctr(s_episode[e], (uint32_t)t, MLG_PURPOSE_RAND, (uint32_t)n));
                        act = random_available(av, A, r2);
                    }
                }
                s_pact[e * N + n] = act;
                bt.actions[bt_off] = act;
                if (bt.full_write)
                    for (int k = 0; k < A; ++k) bt.actions_onehot[bt_off * A + k] = k == act ? 1.0f : 0.0f;
                else
                    bt.actions_onehot[bt_off * A + act] = 1.0f;
            }
        }
        MLG_STAMP(0);
        __syncthreads();
        MLG_STAMP(1);
        // ================= env phase (status 0 envs) ===========================================
        for (int i = tid; i < RE * U; i += nthr) {
            const int e = i / U, u = i % U;
            if (s_status[e] != 0) continue;
            const int ag = SS.agent[u];
            s_act[e * U + u] = env_exec_action(T, s_x + e * U, s_y + e * U, s_hp + e * U, u,
                                               ag ? (int64_t)s_pact[e * N + ag - 1] : 0);
        }
        __syncthreads();
        MLG_STAMP(2);
        for (int i = tid; i < RE * U; i += nthr) {
            const int e = i / U, j = i % U;
            if (s_status[e] != 0) continue;
            s_nhp[e * U + j] = env_resolve_hp(T, s_act + e * U, s_hp + e * U, j);
            if (s_hp[e * U + j] > 0) env_apply_move(s_act[e * U + j], &s_x[e * U + j], &s_y[e * U + j]);
        }
        __syncthreads();
        MLG_STAMP(3);
        for (int e = tid; e < RE; e += nthr) {
            const int b = e0 + e;
            const int status = s_status[e];
            s_stepped[e] = 0;
            if (status == 2) continue;
            for (int n = 0; n < N; ++n) s_prev[e * N + n] = s_pact[e * N + n];
            if (status == 1) {  // final action recorded; env done (parallel_stepper.py:153)
                s_status[e] = 2;
                if (bt.full_write) {
                    bt.reward[(int64_t)s_slot[e] * T1 + t] = 0.f;
                    bt.terminated[(int64_t)s_slot[e] * T1 + t] = 0;
                }
                continue;
            }
            int alive[2] = {0, 0}, lost[2] = {0, 0}, kills[2] = {0, 0};
            for (int j = 0; j < U; ++j) {
                const int tm = SS.team[j];
                const int h0 = s_hp[e * U + j], h1 = s_nhp[e * U + j];
                if (h0 > 0) {
                    lost[tm] += h0 - h1 > 0 ? h0 - h1 : 0;
                    if (h1 == 0) kills[1 - tm] += 1;
                }
                if (h1 > 0) alive[tm] += 1;
                s_hp[e * U + j] = h1;
            }
            const int done = alive[0] == 0 || alive[1] == 0 || t + 1 >= spec.episode_limit;
            int won[2];
            won[0] = alive[1] == 0 && alive[0] > 0;
            won[1] = alive[0] == 0 && alive[1] > 0;
            const int pt = spec.policy_team;
            const int r_int = lost[1 - pt] + 10 * kills[pt] + 200 * won[pt];
            const float r = (float)r_int * 0.0625f;
            bt.reward[(int64_t)s_slot[e] * T1 + t] = r;
            bt.terminated[(int64_t)s_slot[e] * T1 + t] = (uint8_t)done;
            bt.filled[(int64_t)s_slot[e] * T1 + t + 1] = 1;
            s_ret[e] += r;
            s_stepped[e] = 1;
            if (done) {
                s_status[e] = 1;
                s_len[e] = t + 1;
                info.won[2 * b] = won[pt];
                info.won[2 * b + 1] = won[1 - pt];
                info.draw[b] = !won[0] && !won[1];
            }
        }
        __syncthreads();
        MLG_STAMP(4);
        // observation at t + 1 for envs that stepped (incl. those that just terminated)
        for (int i = tid; i < RE * N * U; i += nthr) {
            const int e = i / (N * U), r = i % (N * U);
            if (!s_stepped[e]) continue;
            write_obs_item(T, spec, s_x + e * U, s_y + e * U, s_hp + e * U,
                           bt.obs + ((int64_t)s_slot[e] * T1 + t + 1) * N * DO, r / U, r % U, inv_p);
        }
        for (int i = tid; i < RE * U; i += nthr) {
            const int e = i / U, j = i % U;
            if (!s_stepped[e]) continue;
            float o[6];
            env_state_feat(T, s_x + e * U, s_y + e * U, s_hp + e * U, j, inv_p, o);
            float* dst = bt.state + ((int64_t)s_slot[e] * T1 + t + 1) * S + j * 6;
#pragma unroll
            for (int f = 0; f < 6; ++f) dst[f] = o[f];
        }
        for (int i = tid; i < RE * N * A; i += nthr) {
            const int e = i / (N * A), r = i % (N * A);
            if (!s_stepped[e]) continue;
            bt.avail[((int64_t)s_slot[e] * T1 + t + 1) * N * A + r] =
                env_avail_one(T, s_x + e * U, s_y + e * U, s_hp + e * U, spec.agent_unit[r / A], r % A);
        }
        // full-write mode: slot t+1 of envs that are done (t+1 > episode length) gets zeros
        if (bt.full_write && t + 1 < T1) zero_slots(bt, s_slot, s_status, s_stepped, e0, B, t + 1, t + 2, N, A, S, DO);
        if (tid == 0) {
            int any = 0;
            for (int e = 0; e < RE; ++e) any |= s_status[e] < 2;
            s_any = any;
        }
        __syncthreads();
        MLG_STAMP(5);
        last_t = t;
        if (!s_any) break;
    }
#ifdef MLG_STAMPS
    if (lane == 0 && g_mlg_stamps) {
        unsigned long long* o = g_mlg_stamps + ((int64_t)blockIdx.x * 8 + wave) * 8;
        for (int k = 0; k < 6; ++k) o[k] = st_acc[k];
        o[6] = __builtin_amdgcn_s_memtime() - st_begin;
        o[7] = 1;
    }
#endif
    // full-write mode: the remaining slots of every env (all of them are done here)
    for (int e = tid; e < RE; e += nthr) s_stepped[e] = 0;
    __syncthreads();
    if (bt.full_write && last_t + 2 < T1) zero_slots(bt, s_slot, s_status, s_stepped, e0, B, last_t + 2, T1, N, A, S, DO);
    // ---- per-env summary + env state write-back ----
    for (int e = tid; e < RE; e += nthr) {
        const int b = e0 + e;
        if (b >= B) continue;
        info.ep_len[b] = s_len[e];
        info.ret[b] = s_ret[e];
        st.t[b] = s_len[e];
    }
    for (int i = tid; i < RE * U; i += nthr) {
        const int e = i / U, u = i % U;
        const int64_t b = e0 + e;
        if (b >= B) continue;
        st.x[b * U + u] = s_x[e * U + u];
        st.y[b * U + u] = s_y[e * U + u];
        st.hp[b * U + u] = s_hp[e * U + u];
    }
}

// ------------------------------------------------------------------------------------------------
// Standalone env kernels (one thread per env) -- the EnvWorker command set for host-side TeamsEnv use
// and for kernel-level parity tests.
__global__ void env_reset_kernel(MlgEnvSpec spec, MlgEnvState st) {
    __shared__ SpecShared SS;
    load_spec_tables(spec, SS);
    const EnvTables T = make_tables(spec, SS);
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= st.B) return;
    const uint32_t ep = st.episode[b];
    st.episode[b] = ep + 1;
    st.t[b] = 0;
    const int U = spec.U;
    for (int u = 0; u < U; ++u) {
        const int tm = SS.team[u];
        env_spawn_unit(T, mlg_env_key(spec.seed, b), ep, u, SS.team_first[tm], SS.team_size[tm], st.x + (int64_t)b * U,
                       st.y + (int64_t)b * U, st.hp + (int64_t)b * U);
    }
}

__global__ void env_step_kernel(MlgEnvSpec spec, MlgEnvState st, const int64_t* __restrict__ actions, float* reward,
                                int32_t* done_out, int32_t* won_out, int32_t* draw_out) {
    __shared__ SpecShared SS;
    __shared__ int s_act[64][MLG_MAXU], s_nhp[64][MLG_MAXU];
    load_spec_tables(spec, SS);
    const EnvTables T = make_tables(spec, SS);
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= st.B) return;
    const int U = spec.U, N = spec.n_agents;
    int* x = st.x + (int64_t)b * U;
    int* y = st.y + (int64_t)b * U;
    int* hp = st.hp + (int64_t)b * U;
    int* act = s_act[threadIdx.x];
    int* nhp = s_nhp[threadIdx.x];
    for (int u = 0; u < U; ++u) {
        const int ag = SS.agent[u];
        act[u] = env_exec_action(T, x, y, hp, u, ag ? actions[(int64_t)b * N + ag - 1] : 0);
    }
    for (int j = 0; j < U; ++j) nhp[j] = env_resolve_hp(T, act, hp, j);
    for (int j = 0; j < U; ++j)
        if (hp[j] > 0) env_apply_move(act[j], &x[j], &y[j]);
    int alive[2] = {0, 0}, lost[2] = {0, 0}, kills[2] = {0, 0};
    for (int j = 0; j < U; ++j) {
        const int tm = SS.team[j];
        if (hp[j] > 0) {
            lost[tm] += hp[j] - nhp[j] > 0 ? hp[j] - nhp[j] : 0;
            if (nhp[j] == 0) kills[1 - tm] += 1;
        }
        if (nhp[j] > 0) alive[tm] += 1;
        hp[j] = nhp[j];
    }
    const int t = st.t[b];
    const int done = alive[0] == 0 || alive[1] == 0 || t + 1 >= spec.episode_limit;
    st.t[b] = t + 1;
    int won[2];
    won[0] = alive[1] == 0 && alive[0] > 0;
    won[1] = alive[0] == 0 && alive[1] > 0;
    // reward list: one entry per policy (non-scripted) team in plan order (policy team first)
    int k = 0;
    for (int tm = 0; tm < 2; ++tm) {
        if (spec.scripted[tm]) continue;
        const int r_int = lost[1 - tm] + 10 * kills[tm] + 200 * won[tm];
        reward[(int64_t)b * spec.n_policy_teams + k] = (float)r_int * 0.0625f;
        ++k;
    }
    done_out[b] = done;
    won_out[2 * b] = won[spec.policy_team];
    won_out[2 * b + 1] = won[1 - spec.policy_team];
    draw_out[b] = done && !won[0] && !won[1];
}

__global__ void env_observe_kernel(MlgEnvSpec spec, MlgEnvState st, float* obs, float* state, int32_t* avail) {
    __shared__ SpecShared SS;
    load_spec_tables(spec, SS);
    const EnvTables T = make_tables(spec, SS);
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= st.B) return;
    const int U = spec.U, N = spec.n_agents, A = spec.n_actions;
    const int* x = st.x + (int64_t)b * U;
    const int* y = st.y + (int64_t)b * U;
    const int* hp = st.hp + (int64_t)b * U;
    const float inv_p = 1.0f / (float)pow2_at_least(spec.grid);
    for (int a = 0; a < N; ++a)
        for (int j = 0; j < U; ++j) env_obs_feat(T, x, y, hp, spec.agent_unit[a], j, inv_p, obs + (((int64_t)b * N + a) * U + j) * 8);
    for (int j = 0; j < U; ++j) env_state_feat(T, x, y, hp, j, inv_p, state + ((int64_t)b * U + j) * 6);
    for (int a = 0; a < N; ++a)
        for (int k = 0; k < A; ++k) avail[((int64_t)b * N + a) * A + k] = env_avail_one(T, x, y, hp, spec.agent_unit[a], k);
}

int check_spec(const MlgEnvSpec* s) {
    MLG_REQUIRE(s != nullptr, "null spec");
    MLG_REQUIRE(s->U >= 2 && s->U <= MLG_MAXU, "spec.U=%d out of range [2, %d]", s->U, MLG_MAXU);
    MLG_REQUIRE(s->n_agents >= 1 && s->n_agents <= s->U, "spec.n_agents=%d invalid", s->n_agents);
    MLG_REQUIRE(s->n_actions == MLG_ACT_BASE + s->U, "spec.n_actions must be 5+U");
    MLG_REQUIRE(s->grid >= 2 && s->grid <= 4096, "spec.grid=%d invalid", s->grid);
    MLG_REQUIRE(s->episode_limit >= 1 && s->episode_limit < 65535, "spec.episode_limit invalid");
    MLG_REQUIRE(s->policy_team == 0 || s->policy_team == 1, "spec.policy_team invalid");
    for (int u = 0; u < s->U; ++u) {
        MLG_REQUIRE(s->team[u] == 0 || s->team[u] == 1, "unit %d team invalid", u);
        MLG_REQUIRE(s->role[u] >= 0 && s->role[u] <= 2, "unit %d role invalid", u);
        MLG_REQUIRE(s->melee[u] == 0 || s->melee[u] == 1, "unit %d attack type invalid", u);
    }
    for (int a = 0; a < s->n_agents; ++a)
        MLG_REQUIRE(s->agent_unit[a] >= 0 && s->agent_unit[a] < s->U, "agent %d unit invalid", a);
    return 0;
}

int check_state(const MlgEnvState* st) {
    MLG_REQUIRE(st && st->x && st->y && st->hp && st->t && st->episode, "env state has null pointers");
    MLG_REQUIRE(st->B >= 1, "env state B=%d", st->B);
    return 0;
}

constexpr int LDS_LIMIT_BYTES = 160 * 1024;

template <int H, int TPW, bool WLDS>
int launch_rollout_t(int grid, int threads, hipStream_t s, const MlgEnvSpec& spec, const MlgEnvState& st,
                     const AgentLayout& L, const float* P, const MlgBatch& bt, const MlgRunInfo& info, float eps, int tm,
                     const RolloutLds& lay) {
    const size_t bytes = (size_t)lay.total * 4;
    auto kern = rollout_kernel<H, TPW, WLDS>;
    if (bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)bytes);
        if (e != hipSuccess) return mlg::fail("rollout: LDS attribute (%zu B): %s", bytes, hipGetErrorString(e));
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), bytes, s, spec, st, L, P, bt, info, eps, tm, lay);
    return 0;
}

template <int H, int TPW>
int launch_rollout(int grid, int threads, hipStream_t s, const MlgEnvSpec& spec, const MlgEnvState& st,
                   const AgentLayout& L, const float* P, const MlgBatch& bt, const MlgRunInfo& info, float eps, int tm) {
    RolloutLds lay = make_rollout_lds(L, spec.U, spec.n_agents, true);
    if (lay.total * 4 <= LDS_LIMIT_BYTES && !getenv("MLG_ROLLOUT_GLOBAL_WEIGHTS"))
        return launch_rollout_t<H, TPW, true>(grid, threads, s, spec, st, L, P, bt, info, eps, tm, lay);
    lay = make_rollout_lds(L, spec.U, spec.n_agents, false);
    return launch_rollout_t<H, TPW, false>(grid, threads, s, spec, st, L, P, bt, info, eps, tm, lay);
}

}  // namespace

int check_agent_dims(const MlgAgentDims* d);  // agent.hip

// ---- zero a range of EpisodeBatch slots (ring mode pre-fill): one launch over every key ----------------
struct ZeroJobs {
    unsigned char* base[16];
    int64_t begin[16], end[16];  // byte ranges
    int64_t words0[17];          // prefix sums of 16-byte words of each job's aligned interior
    int n;
};

__global__ void zero_ranges_kernel(ZeroJobs J) {
    const int64_t total = J.words0[J.n];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int j = 0;
        while (j + 1 < J.n && J.words0[j + 1] <= i) ++j;
        const int64_t a0 = (J.begin[j] + 15) & ~int64_t(15);
        *reinterpret_cast<uint4*>(J.base[j] + a0 + (i - J.words0[j]) * 16) = make_uint4(0, 0, 0, 0);
    }
    // unaligned heads / tails (< 16 bytes each): one thread per job
    if (blockIdx.x == 0 && threadIdx.x < J.n) {
        const int j = threadIdx.x;
        const int64_t a0 = (J.begin[j] + 15) & ~int64_t(15), a1 = J.end[j] & ~int64_t(15);
        if (a0 >= a1) {
            for (int64_t b = J.begin[j]; b < J.end[j]; ++b) J.base[j][b] = 0;
        } else {
            for (int64_t b = J.begin[j]; b < a0; ++b) J.base[j][b] = 0;
            for (int64_t b = a1; b < J.end[j]; ++b) J.base[j][b] = 0;
        }
    }
}

extern "C" int mlg_zero_slots_bytes(const MlgBatch* bt, const int64_t* slot_bytes /*[8]*/, int32_t slot0, int32_t count,
                                    int32_t ring_size, void* stream) {
    MLG_REQUIRE(bt && slot_bytes, "zero_slots: null argument");
    MLG_REQUIRE(ring_size >= 1 && count >= 0 && count <= ring_size && slot0 >= 0 && slot0 < ring_size,
                "zero_slots: bad range (slot0=%d count=%d ring=%d)", slot0, count, ring_size);
    void* ptrs[8] = {bt->state, bt->obs, bt->actions, bt->avail, bt->reward, bt->terminated, bt->actions_onehot,
                     bt->filled};
    ZeroJobs J;
    J.n = 0;
    J.words0[0] = 0;
    const int first = (slot0 + count <= ring_size) ? count : ring_size - slot0;
    const int second = count - first;
    for (int k = 0; k < 8; ++k) {
        MLG_REQUIRE(ptrs[k] != nullptr && slot_bytes[k] > 0, "zero_slots: key %d missing", k);
        for (int part = 0; part < 2; ++part) {
            const int s0 = part == 0 ? slot0 : 0, n = part == 0 ? first : second;
            if (n <= 0) continue;
            J.base[J.n] = reinterpret_cast<unsigned char*>(ptrs[k]);
            J.begin[J.n] = (int64_t)s0 * slot_bytes[k];
            J.end[J.n] = (int64_t)(s0 + n) * slot_bytes[k];
            const int64_t a0 = (J.begin[J.n] + 15) & ~int64_t(15), a1 = J.end[J.n] & ~int64_t(15);
            J.words0[J.n + 1] = J.words0[J.n] + (a1 > a0 ? (a1 - a0) / 16 : 0);
            ++J.n;
        }
    }
    if (J.n == 0) return 0;
    hipLaunchKernelGGL(zero_ranges_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, J);
    return mlg::check_launch("zero_ranges_kernel");
}

extern "C" int mlg_debug_set_stamps(void* ptr) {
#ifdef MLG_STAMPS
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_mlg_stamps), &ptr, sizeof(ptr));
    if (e != hipSuccess) return mlg::fail("set stamps: %s", hipGetErrorString(e));
    return 0;
#else
    (void)ptr;
    return mlg::fail("not a stamps build (-DMLG_STAMPS)");
#endif
}

extern "C" int mlg_env_reset(const MlgEnvSpec* spec, MlgEnvState* st, void* stream) {
    if (check_spec(spec) || check_state(st)) return 1;
    hipLaunchKernelGGL(env_reset_kernel, dim3((st->B + 63) / 64), dim3(64), 0, (hipStream_t)stream, *spec, *st);
    return mlg::check_launch("env_reset_kernel");
}

extern "C" int mlg_env_step(const MlgEnvSpec* spec, MlgEnvState* st, const int64_t* actions, float* reward,
                            int32_t* done, int32_t* won, int32_t* draw, void* stream) {
    if (check_spec(spec) || check_state(st)) return 1;
    MLG_REQUIRE(actions && reward && done && won && draw, "env_step: null output pointer");
    hipLaunchKernelGGL(env_step_kernel, dim3((st->B + 63) / 64), dim3(64), 0, (hipStream_t)stream, *spec, *st, actions,
                       reward, done, won, draw);
    return mlg::check_launch("env_step_kernel");
}

extern "C" int mlg_env_observe(const MlgEnvSpec* spec, const MlgEnvState* st, float* obs, float* state, int32_t* avail,
                               void* stream) {
    if (check_spec(spec) || check_state(st)) return 1;
    MLG_REQUIRE(obs && state && avail, "env_observe: null output pointer");
    hipLaunchKernelGGL(env_observe_kernel, dim3((st->B + 63) / 64), dim3(64), 0, (hipStream_t)stream, *spec, *st, obs,
                       state, avail);
    return mlg::check_launch("env_observe_kernel");
}

extern "C" int mlg_rollout(const MlgEnvSpec* spec, MlgEnvState* st, const MlgAgentDims* dims, const float* packed,
                           MlgBatch* batch, MlgRunInfo* info, float epsilon, int32_t test_mode, void* stream) {
    if (check_spec(spec) || check_state(st) || check_agent_dims(dims)) return 1;
    MLG_REQUIRE(packed && batch && info, "rollout: null pointer");
    MLG_REQUIRE(batch->state && batch->obs && batch->actions && batch->avail && batch->reward && batch->terminated &&
                    batch->actions_onehot && batch->filled,
                "rollout: batch has null tensors");
    MLG_REQUIRE(info->ep_len && info->ret && info->won && info->draw, "rollout: run info has null tensors");
    MLG_REQUIRE(batch->B == st->B, "rollout: batch B=%d != env B=%d", batch->B, st->B);
    MLG_REQUIRE(batch->T1 == spec->episode_limit + 1, "rollout: batch T1=%d != episode_limit+1=%d", batch->T1,
                spec->episode_limit + 1);
    MLG_REQUIRE(dims->n_agents == spec->n_agents && dims->n_actions == spec->n_actions && dims->d_obs == 8 * spec->U,
                "rollout: agent dims do not match env spec (N=%d/%d A=%d/%d d_obs=%d/%d)", dims->n_agents,
                spec->n_agents, dims->n_actions, spec->n_actions, dims->d_obs, 8 * spec->U);
    const AgentLayout L = make_agent_layout(*dims);
    const int tiles = (RE * spec->n_agents + 15) / 16;
    const int W = tiles < 8 ? tiles : 8;
    const int tpw = (tiles + W - 1) / W;
    const int grid = (st->B + RE - 1) / RE;
    const int threads = W * 64;
    hipStream_t s = (hipStream_t)stream;
    const float eps = test_mode ? 0.f : epsilon;
    int rc = 0;
#define MLG_RO(HH, TT) rc = launch_rollout<HH, TT>(grid, threads, s, *spec, *st, L, packed, *batch, *info, eps, test_mode)
    if (dims->hidden == 64) {
        if (tpw == 1) MLG_RO(64, 1);
        else if (tpw == 2) MLG_RO(64, 2);
        else if (tpw == 3) MLG_RO(64, 3);
        else MLG_RO(64, 4);
    } else if (dims->hidden == 32) {
        if (tpw == 1) MLG_RO(32, 1);
        else if (tpw == 2) MLG_RO(32, 2);
        else if (tpw == 3) MLG_RO(32, 3);
        else MLG_RO(32, 4);
    } else if (dims->hidden == 128) {
        if (tpw == 1) MLG_RO(128, 1);
        else if (tpw == 2) MLG_RO(128, 2);
        else if (tpw == 3) MLG_RO(128, 3);
        else MLG_RO(128, 4);
    } else {
        return mlg::fail("rollout: rnn_hidden_dim=%d unsupported (32, 64, 128)", dims->hidden);
    }
#undef MLG_RO
    if (rc) return rc;
    return mlg::check_launch("rollout_kernel");
}
