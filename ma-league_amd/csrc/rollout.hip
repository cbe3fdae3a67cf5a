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
#include <cstring>

#include "agent_device.h"
#include "mlg_host.h"

#ifdef MLG_STAMPS
// Diagnostic build only (-DMLG_STAMPS, libmaleague_stamps.so): per-wave cycle counts of the rollout phases,
// written to g_mlg_stamps[block][wave][32] (slots 0..29 phases, 30 total, 31 = 1).
__device__ unsigned long long* g_mlg_stamps = nullptr;
struct Stamps {
    unsigned long long acc[30], last, begin, tstep;
    __device__ void init() {
        for (int k = 0; k < 30; ++k) acc[k] = 0;
        last = begin = tstep = __builtin_amdgcn_s_memtime();
    }
    // step trace (wave 0): cycles of step t-1 and running envs of step t, after the phase slots of the grid
    __device__ void step(int t, int nrun) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        if (g_mlg_stamps && threadIdx.x == 0 && t < 128)
            g_mlg_stamps[(int64_t)gridDim.x * 8 * 32 + (int64_t)blockIdx.x * 128 + t] = ((now - tstep) << 8) | (unsigned)nrun;
        tstep = now;
#ifdef MLG_STAMPS_LOWRUN
        on = nrun <= MLG_STAMPS_LOWRUN;
#endif
#ifdef MLG_STAMPS_MINRUN  // phase slots count only the steps with >= k running envs (full-occupancy breakdown)
        on = nrun >= MLG_STAMPS_MINRUN;
#endif
#ifdef MLG_STAMPS_TIMELINE
        on = nrun == 1 && !seen;
        seen = seen || on;
#endif
    }
    bool on = true;  // -DMLG_STAMPS_LOWRUN=k: phase slots count only the steps with <= k running envs
    bool seen = false;
    __device__ void mark(int k) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
#ifdef MLG_STAMPS_TIMELINE  // slot k = cycles from the start of the first one-env step to mark k
        if (on) acc[k] = now - tstep;
#else
        if (on) acc[k] += now - last;
#endif
        last = now;
    }
    __device__ void flush() {
        if ((threadIdx.x & 63) || !g_mlg_stamps) return;
        unsigned long long* o = g_mlg_stamps + ((int64_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * 32;
        for (int k = 0; k < 30; ++k) o[k] = acc[k];
        o[30] = __builtin_amdgcn_s_memtime() - begin;
        o[31] = 1;
    }
};
#else
struct Stamps {
    __device__ void init() {}
    __device__ void mark(int) {}
    __device__ void step(int, int) {}
    __device__ void flush() {}
};
#endif

namespace {

constexpr int RE = 16;  // envs per workgroup

struct SpecShared {
    int team[MLG_MAXU], role[MLG_MAXU], melee[MLG_MAXU], agent[MLG_MAXU];
    int aunit[MLG_MAXU];  // unit of agent a
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
    for (int a = tid; a < spec.n_agents; a += blockDim.x) {
        s.agent[spec.agent_unit[a]] = a + 1;
        s.aunit[a] = spec.agent_unit[a];
    }
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

// ---- per-workgroup env bookkeeping shared by both rollout kernels --------------------------------
// LDS pointers of the RE envs a workgroup owns. lobs/lavail (v2 only, else nullptr) mirror the obs and
// avail rows the agent phase reads, so the cell never reads back what the env phase wrote to HBM.
struct RoEnv {
    int *x, *y, *hp, *nhp, *act, *pact, *prev, *status, *stepped, *len, *slot, *list, *misc;
    int* slot2;  // batch slot of the away side (self-play, v1 only)
    uint32_t* episode;
    float *ret, *ret2;  // episode return of side 0 (home / policy team) and side 1 (away)
    float* lobs;
    int32_t* lavail;
    int ldo;
};

// Dynamic-LDS carve of the env part (4-byte words).
struct RoEnvLds {
    int32_t spec, x, y, hp, nhp, act, pact, prev, status, stepped, len, episode, ret, slot, list, misc, slot2, ret2;
};

__host__ __device__ constexpr int64_t ro_take(int64_t& o, int64_t n) {
    const int64_t v = o;
    o += mlg_align4(n);
    return v;
}

// The fields the v2-structure env lanes use (status, episode, slot, pending / previous actions); the others alias
// offset 0 and are never dereferenced by those kernels.
__host__ __device__ constexpr RoEnvLds make_env_lds_v2(int64_t& o, int n_agents, int re) {
    RoEnvLds r{};
    r.spec = ro_take(o, (int64_t)(sizeof(SpecShared) / 4));
    r.pact = ro_take(o, (int64_t)re * n_agents);
    r.prev = ro_take(o, (int64_t)re * n_agents);
    r.status = ro_take(o, re);
    r.episode = ro_take(o, re);
    r.slot = ro_take(o, re);
    return r;
}

__host__ __device__ constexpr RoEnvLds make_env_lds(int64_t& o, int U, int n_agents, int re = RE) {
    RoEnvLds r{};
    r.spec = ro_take(o, (int64_t)(sizeof(SpecShared) / 4));
    const int64_t eu = (int64_t)re * U;
    r.x = ro_take(o, eu);
    r.y = ro_take(o, eu);
    r.hp = ro_take(o, eu);
    r.nhp = ro_take(o, eu);
    r.act = ro_take(o, eu);
    r.pact = ro_take(o, (int64_t)re * n_agents);
    r.prev = ro_take(o, (int64_t)re * n_agents);
    r.status = ro_take(o, re);
    r.stepped = ro_take(o, re);
    r.len = ro_take(o, re);
    r.episode = ro_take(o, re);
    r.ret = ro_take(o, re);
    r.slot = ro_take(o, re);
    r.list = ro_take(o, re);
    r.misc = ro_take(o, 4);  // [0] any env running, [1] number of running envs
    r.slot2 = ro_take(o, re);
    r.ret2 = ro_take(o, re);
    return r;
}

__device__ inline RoEnv env_view(int* smem, const RoEnvLds& l) {
    RoEnv R;
    R.x = smem + l.x;
    R.y = smem + l.y;
    R.hp = smem + l.hp;
    R.nhp = smem + l.nhp;
    R.act = smem + l.act;
    R.pact = smem + l.pact;
    R.prev = smem + l.prev;
    R.status = smem + l.status;
    R.stepped = smem + l.stepped;
    R.len = smem + l.len;
    R.slot = smem + l.slot;
    R.list = smem + l.list;
    R.misc = smem + l.misc;
    R.episode = reinterpret_cast<uint32_t*>(smem + l.episode);
    R.ret = reinterpret_cast<float*>(smem + l.ret);
    R.slot2 = smem + l.slot2;
    R.ret2 = reinterpret_cast<float*>(smem + l.ret2);
    R.lobs = nullptr;
    R.lavail = nullptr;
    R.ldo = 0;
    return R;
}

// Policy sides of a rollout. ns = 1: one MAC acts for the policy team (ParallelStepper). ns = 2: self-play
// (self_play_parallel_stepper.py:97-108): agents [0, nh) are the home team and act with P[0] into bt[0],
// agents [nh, 2 nh) the away team with P[1] into bt[1]; stepper_utils.build_pre_transition_data
// (stepper_utils.py:4-24) splits obs / avail the same way, state goes to both batches.
struct Sides {
    MlgBatch bt[2];
    const float* P[2];
    float eps[2];
    int ns, nh;
};

// Field selects instead of dynamic indexing: keeps the kernel-argument struct in SGPRs (no scratch copy).
__device__ __forceinline__ MlgBatch side_batch(const Sides& sd, int side) { return side ? sd.bt[1] : sd.bt[0]; }
__device__ __forceinline__ int side_slot(const RoEnv& R, int side, int e) { return side ? R.slot2[e] : R.slot[e]; }

// obs/state/avail of batch time index t for the envs selected by `sel` (0: not done at reset, 1: stepped).
__device__ void ro_observe(const EnvTables& T, const MlgEnvSpec& spec, const RoEnv& R, const Sides& sd, int t,
                           bool stepped_only, float inv_p, Stamps& sp) {
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int U = T.U, N = spec.n_agents, A = spec.n_actions, S = 6 * U, DO = 8 * U, T1 = sd.bt[0].T1, nh = sd.nh;
    auto on = [&](int e) { return stepped_only ? R.stepped[e] != 0 : R.status[e] != 2; };
    for (int i = tid; i < RE * N * U; i += nthr) {
        const int e = i / (N * U), r = i % (N * U);
        if (!on(e)) continue;
        const int a = r / U, j = r % U;
        const int side = a >= nh, ln = a - side * nh;
        float o[8];
        env_obs_feat(T, R.x + e * U, R.y + e * U, R.hp + e * U, spec.agent_unit[a], j, inv_p, o);
        const floatx4 lo{o[0], o[1], o[2], o[3]}, hi{o[4], o[5], o[6], o[7]};
        float* dst = side_batch(sd, side).obs + (((int64_t)side_slot(R, side, e) * T1 + t) * nh + ln) * DO + j * 8;
        *reinterpret_cast<floatx4*>(dst) = lo;
        *reinterpret_cast<floatx4*>(dst + 4) = hi;
        if (R.lobs) {
            float* l = R.lobs + (e * N + a) * R.ldo + j * 8;
            *reinterpret_cast<floatx4*>(l) = lo;
            *reinterpret_cast<floatx4*>(l + 4) = hi;
        }
    }
    sp.mark(7);
    for (int i = tid; i < RE * U; i += nthr) {
        const int e = i / U, j = i % U;
        if (!on(e)) continue;
        float o[6];
        env_state_feat(T, R.x + e * U, R.y + e * U, R.hp + e * U, j, inv_p, o);
        for (int side = 0; side < sd.ns; ++side) {
            float* dst = side_batch(sd, side).state + ((int64_t)side_slot(R, side, e) * T1 + t) * S + j * 6;
#pragma unroll
            for (int f = 0; f < 6; ++f) dst[f] = o[f];
        }
    }
    sp.mark(8);
    for (int i = tid; i < RE * N * A; i += nthr) {
        const int e = i / (N * A), r = i % (N * A);
        if (!on(e)) continue;
        const int a = r / A, side = a >= nh;
        const int v = env_avail_one(T, R.x + e * U, R.y + e * U, R.hp + e * U, spec.agent_unit[a], r % A);
        side_batch(sd, side).avail[((int64_t)side_slot(R, side, e) * T1 + t) * nh * A + r - side * nh * A] = v;
        if (R.lavail) R.lavail[e * N * A + r] = v;
    }
    sp.mark(9);
}

__device__ __forceinline__ int ring_slot_of(const MlgBatch& b, int env) {
    return b.ring_size > 0 ? (b.ring_slot0 + env) % b.ring_size : env;
}

// Reset of the RE envs (parallel_stepper.py:82-104; env_worker_process.py:54-60) + observation at t = 0.
__device__ void ro_reset(const EnvTables& T, const SpecShared& SS, const MlgEnvSpec& spec, const MlgEnvState& st,
                         const RoEnv& R, const Sides& sd, int e0, float inv_p) {
    const int tid = threadIdx.x, nthr = blockDim.x, U = T.U, B = sd.bt[0].B;
    for (int e = tid; e < RE; e += nthr) {
        const int b = e0 + e;
        R.len[e] = 0;
        R.ret[e] = 0.f;
        R.ret2[e] = 0.f;
        R.stepped[e] = 0;
        if (b < B) {
            const uint32_t ep = st.episode[b];
            st.episode[b] = ep + 1;
            R.episode[e] = ep;
            R.status[e] = 0;
            R.slot[e] = ring_slot_of(sd.bt[0], b);
            R.slot2[e] = ring_slot_of(sd.bt[1], b);
            for (int side = 0; side < sd.ns; ++side) {
                const MlgBatch bt = side_batch(sd, side);
                bt.filled[(int64_t)side_slot(R, side, e) * bt.T1] = 1;
            }
        } else {
            R.status[e] = 2;
        }
    }
    __syncthreads();
    for (int i = tid; i < RE * U; i += nthr) {
        const int e = i / U, u = i % U;
        if (R.status[e] == 2) continue;
        const int tm = SS.team[u];
        env_spawn_unit(T, mlg_env_key(spec.seed, e0 + e), R.episode[e], u, SS.team_first[tm], SS.team_size[tm],
                       R.x + e * U, R.y + e * U, R.hp + e * U);
    }
    __syncthreads();
    Stamps none;
    ro_observe(T, spec, R, sd, 0, false, inv_p, none);
}

// Running-env list (status < 2, ascending) and count; single thread, caller syncs.
__device__ inline void ro_list_running(const RoEnv& R) {
    int n = 0;
    for (int e = 0; e < RE; ++e)
        if (R.status[e] < 2) R.list[n++] = e;
    R.misc[0] = n > 0;
    R.misc[1] = n;
}

// Env phase of step t for the running envs (env_worker_process.py:32-53 batched): executed actions
// (policy or scripted AI), simultaneous resolution, per-env reward / termination, then obs of t + 1.
// Side s receives the reward of its own team (self-play: reward = (home, away), self_play_parallel_stepper.py:159).
__device__ void ro_env_step(const EnvTables& T, const SpecShared& SS, const MlgEnvSpec& spec, const RoEnv& R,
                            const Sides& sd, const MlgRunInfo& info, int e0, int t, float inv_p, Stamps& sp) {
    const int tid = threadIdx.x, nthr = blockDim.x, U = T.U, N = spec.n_agents, T1 = sd.bt[0].T1;
    for (int i = tid; i < RE * U; i += nthr) {
        const int e = i / U, u = i % U;
        if (R.status[e] != 0) continue;
        const int ag = SS.agent[u];
        R.act[e * U + u] = env_exec_action(T, R.x + e * U, R.y + e * U, R.hp + e * U, u,
                                           ag ? (int64_t)R.pact[e * N + ag - 1] : 0);
    }
    sp.mark(4);
    __syncthreads();
    for (int i = tid; i < RE * U; i += nthr) {
        const int e = i / U, j = i % U;
        if (R.status[e] != 0) continue;
        R.nhp[e * U + j] = env_resolve_hp(T, R.act + e * U, R.hp + e * U, j);
        if (R.hp[e * U + j] > 0) env_apply_move(R.act[e * U + j], &R.x[e * U + j], &R.y[e * U + j]);
    }
    sp.mark(5);
    __syncthreads();
    const int pt = spec.policy_team;  // team of side 0; side 1 (self-play) is the other plan team
    for (int e = tid; e < RE; e += nthr) {
        const int b = e0 + e;
        const int status = R.status[e];
        R.stepped[e] = 0;
        if (status == 2) continue;
        for (int n = 0; n < N; ++n) R.prev[e * N + n] = R.pact[e * N + n];
        if (status == 1) {  // final action recorded; env done (parallel_stepper.py:153)
            R.status[e] = 2;
            for (int side = 0; side < sd.ns; ++side) {
                const MlgBatch bt = side_batch(sd, side);
                if (bt.full_write) {
                    bt.reward[(int64_t)side_slot(R, side, e) * T1 + t] = 0.f;
                    bt.terminated[(int64_t)side_slot(R, side, e) * T1 + t] = 0;
                }
            }
            continue;
        }
        int alive[2] = {0, 0}, lost[2] = {0, 0}, kills[2] = {0, 0};
        for (int j = 0; j < U; ++j) {
            const int tm = SS.team[j];
            const int h0 = R.hp[e * U + j], h1 = R.nhp[e * U + j];
            if (h0 > 0) {
                lost[tm] += h0 - h1 > 0 ? h0 - h1 : 0;
                if (h1 == 0) kills[1 - tm] += 1;
            }
            if (h1 > 0) alive[tm] += 1;
            R.hp[e * U + j] = h1;
        }
        const int done = alive[0] == 0 || alive[1] == 0 || t + 1 >= spec.episode_limit;
        int won[2];
        won[0] = alive[1] == 0 && alive[0] > 0;
        won[1] = alive[0] == 0 && alive[1] > 0;
        for (int side = 0; side < sd.ns; ++side) {
            const int tm = side ? 1 - pt : pt;
            const float r = (float)(lost[1 - tm] + 10 * kills[tm] + 200 * won[tm]) * 0.0625f;
            const MlgBatch bt = side_batch(sd, side);
            const int64_t sl = (int64_t)side_slot(R, side, e) * T1 + t;
            bt.reward[sl] = r;
            bt.terminated[sl] = (uint8_t)done;
            bt.filled[sl + 1] = 1;
            if (side) R.ret2[e] += r;
            else R.ret[e] += r;
        }
        R.stepped[e] = 1;
        if (done) {
            R.status[e] = 1;
            R.len[e] = t + 1;
            info.won[2 * b] = won[pt];
            info.won[2 * b + 1] = won[1 - pt];
            info.draw[b] = !won[0] && !won[1];
        }
    }
    sp.mark(6);
    __syncthreads();
    // observation at t + 1 for envs that stepped (incl. those that just terminated)
    ro_observe(T, spec, R, sd, t + 1, true, inv_p, sp);
}

// Zero every key of slots [t0, t1) of the envs of this workgroup that are done and did not step
// (status 2, or stepped == 0 with status 2 after the final action): the full-write (ring) mode's
// replacement for zero-initialising the EpisodeBatch. Sides in full-write mode only.
__device__ void zero_slots(const Sides& sd, const RoEnv& R, int e0, int t0, int t1, int A, int S, int DO) {
    const int T1 = sd.bt[0].T1, B = sd.bt[0].B, N = sd.nh;
    const int per = S + N * DO + 2 * N * A + 2 * N + 3;  // words per slot (actions/filled are 2 words)
    const int total = sd.ns * RE * (t1 - t0) * per;
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
        const int side = i / (RE * (t1 - t0) * per), ii = i % (RE * (t1 - t0) * per);
        const int e = ii / ((t1 - t0) * per), rem = ii % ((t1 - t0) * per);
        const int t = t0 + rem / per;
        int k = rem % per;
        const MlgBatch bt = side_batch(sd, side);
        if (!bt.full_write || e0 + e >= B || R.status[e] != 2 || R.stepped[e]) continue;
        const int64_t sl = (int64_t)side_slot(R, side, e) * T1 + t;
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

// Per-env summary + env state write-back.
__device__ void ro_finish(const MlgEnvState& st, const RoEnv& R, const Sides& sd, const MlgRunInfo& info, int e0, int B,
                          int U) {
    const int tid = threadIdx.x, nthr = blockDim.x;
    for (int e = tid; e < RE; e += nthr) {
        const int b = e0 + e;
        if (b >= B) continue;
        info.ep_len[b] = R.len[e];
        info.ret[b] = R.ret[e];
        if (info.ret_away) info.ret_away[b] = R.ret2[e];
        st.t[b] = R.len[e];
        for (int side = 0; side < sd.ns; ++side) {  // v1 zeroes every tail row: the slot's extent is L + 1
            const MlgBatch bt = side_batch(sd, side);
            if (bt.full_write && bt.slot_extent) bt.slot_extent[side_slot(R, side, e)] = R.len[e] + 1;
        }
    }
    for (int i = tid; i < RE * U; i += nthr) {
        const int e = i / U, u = i % U;
        const int64_t b = e0 + e;
        if (b >= B) continue;
        st.x[b * U + u] = R.x[e * U + u];
        st.y[b * U + u] = R.y[e * U + u];
        st.hp[b * U + u] = R.hp[e * U + u];
    }
}

// Picks the action of agent a (global index; side a >= nh) from the masked argmax
// (EpsilonGreedyActionSelector.select, action_selectors.py:44-62) and records it: LDS pending action,
// the side's batch actions / actions_onehot. The epsilon RNG stream index is the global agent index.
__device__ __forceinline__ void ro_record_action(const MlgEnvSpec& spec, const RoEnv& R, const Sides& sd, int act,
                                                 const int32_t* av, int e, int a, int b, int t, int test_mode) {
    const int N = spec.n_agents, A = spec.n_actions, nh = sd.nh;
    const int side = a >= nh, ln = a - side * nh;
    const float eps = side ? sd.eps[1] : sd.eps[0];
    if (!test_mode && eps > 0.f) {
        const uint64_t key = mlg_env_key(spec.seed, b);
        const uint64_t r1 = mlg_rng(key, mlg_ctr(R.episode[e], (uint32_t)t, MLG_PURPOSE_EPS, (uint32_t)a));
        if (mlg_u01(r1) < eps) {
            const uint64_t r2 = mlg_rng(key, mlg_ctr(R.episode[e], (uint32_t)t, MLG_PURPOSE_RAND, (uint32_t)a));
            act = random_available(av, A, r2);
        }
    }
    R.pact[e * N + a] = act;
    const MlgBatch bt = side_batch(sd, side);
    const int64_t bt_off = ((int64_t)side_slot(R, side, e) * bt.T1 + t) * nh + ln;
    bt.actions[bt_off] = act;
    if (bt.full_write)
        for (int k = 0; k < A; ++k) bt.actions_onehot[bt_off * A + k] = k == act ? 1.0f : 0.0f;
    else
        bt.actions_onehot[bt_off * A + act] = 1.0f;
}

// ================================================================================================
// v1: generic kernel (any H in {32, 64, 128}, weights in LDS or HBM; the only kernel with self-play sides).
// Workgroup = W waves (W = min(tiles, 8)); wave w owns the 16-row agent tiles w, w + W, ... for the whole
// episode with the GRU hidden state in VGPRs. Tiles never mix sides: side s owns tiles [s tps, (s+1) tps),
// row r of side s = env (r / nh), agent s nh + r % nh.
struct RolloutLds {
    int32_t wts, total;
    RoEnvLds env;
    LdsWeights lw;
    int weights_in_lds;
};

__host__ __device__ inline RolloutLds make_rollout_lds(const AgentLayout& L, int U, int n_agents, bool weights_in_lds) {
    RolloutLds r;
    r.lw = make_lds_weights(L);
    r.weights_in_lds = weights_in_lds;
    int64_t o = 0;
    r.wts = ro_take(o, weights_in_lds ? r.lw.total : 0);
    r.env = make_env_lds(o, U, n_agents);
    r.total = o;
    return r;
}

template <int H, int TPW, bool WLDS>
__global__ void __launch_bounds__(512) rollout_kernel(MlgEnvSpec spec, MlgEnvState st, AgentLayout L, Sides sd,
                                                     MlgRunInfo info, int test_mode, RolloutLds lay) {
    constexpr int HC = H / 16;
    extern __shared__ __attribute__((aligned(16))) int smem[];
    SpecShared& SS = *reinterpret_cast<SpecShared*>(smem + lay.env.spec);
    const RoEnv R = env_view(smem, lay.env);
    const int U = spec.U, N = spec.n_agents, A = spec.n_actions, S = 6 * U, DO = 8 * U, nh = sd.nh;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int lane = tid & 63, wave = tid >> 6, W = nthr >> 6;
    const int e0 = blockIdx.x * RE;
    const int T1 = sd.bt[0].T1;
    const bool any_full_write = sd.bt[0].full_write || (sd.ns > 1 && sd.bt[1].full_write);
    load_spec_tables(spec, SS);
    if (WLDS) load_weights_to_lds(sd.P[0], L, lay.lw, reinterpret_cast<float*>(smem + lay.wts));
    const EnvTables T = make_tables(spec, SS);
    const float inv_p = 1.0f / (float)pow2_at_least(spec.grid);
    ro_reset(T, SS, spec, st, R, sd, e0, inv_p);
    __syncthreads();

    floatx4 h[TPW][HC];
#pragma unroll
    for (int ti = 0; ti < TPW; ++ti)
#pragma unroll
        for (int c = 0; c < HC; ++c) h[ti][c] = floatx4{0.f, 0.f, 0.f, 0.f};
    Stamps sp;
    sp.init();
    const int tps = (RE * nh + 15) / 16, n_tiles = sd.ns * tps;
    const int col = lane & 15, g = lane >> 4;
    const int n_at = L.Ap / 16;
    int last_t = 0;
    for (int t = 0; t < T1; ++t) {
        // ================= agent phase: rows of envs with status 0 (running) or 1 (final action) ======
#pragma unroll
        for (int ti = 0; ti < TPW; ++ti) {
            const int tile = wave + ti * W;
            if (tile >= n_tiles) continue;
            const int side = tile >= tps;
            const int r = (tile - side * tps) * 16 + col;
            const bool in_range = r < RE * nh;
            const int e = in_range ? r / nh : 0, ln = r % nh, a = side * nh + ln;
            const bool valid = in_range && R.status[e] < 2;
            if (!__any(valid)) continue;  // wave-uniform skip of finished tiles
            // Opaque zero offset per tile: stops LICM/CSE from keeping t- and tile-invariant weight loads
            // live across the episode loop in (spilled) registers.
            int zero = 0;
            asm volatile("" : "+s"(zero));
            const WView Wv = WLDS ? lds_view(reinterpret_cast<const float*>(smem + lay.wts) + zero, lay.lw, L)
                                  : global_view((side ? sd.P[1] : sd.P[0]) + zero, L);
            const MlgBatch bt = side_batch(sd, side);
            const int64_t bt_off = valid ? ((int64_t)side_slot(R, side, e) * T1 + t) * nh + ln : 0;
            RowIn in;
            in.x = valid ? bt.obs + bt_off * DO : nullptr;
            in.onehot = nullptr;
            in.prev_action = (valid && t > 0) ? R.prev[e * N + a] : -1;
            in.agent = valid ? ln : 0;
            agent_cell_hidden<H>(Wv, L, in, h[ti], lane);
            const int32_t* av = valid ? bt.avail + bt_off * A : nullptr;
            ArgmaxState as{-INFINITY, 1 << 30};
            for (int at = 0; at < n_at; ++at) {
                const floatx4 q = agent_q_tile<H>(Wv, h[ti], at, lane);
                argmax_accumulate(as, q, av, at, A, lane);
            }
            const int act = argmax_reduce(as);
            if (valid && g == 0) ro_record_action(spec, R, sd, act, av, e, a, e0 + e, t, test_mode);
        }
        sp.mark(0);
        __syncthreads();
        sp.mark(1);
        ro_env_step(T, SS, spec, R, sd, info, e0, t, inv_p, sp);
        // full-write mode: slot t+1 of envs that are done (t+1 > episode length) gets zeros
        if (any_full_write && t + 1 < T1) zero_slots(sd, R, e0, t + 1, t + 2, A, S, DO);
        if (tid == 0) ro_list_running(R);
        __syncthreads();
        sp.mark(10);
        last_t = t;
        if (!R.misc[0]) break;
    }
    sp.flush();
    // full-write mode: the remaining slots of every env (all of them are done here)
    for (int e = tid; e < RE; e += nthr) R.stepped[e] = 0;
    __syncthreads();
    if (any_full_write && last_t + 2 < T1) zero_slots(sd, R, e0, last_t + 2, T1, A, S, DO);
    ro_finish(st, R, sd, info, e0, sd.bt[0].B, U);
}

// Full-write tail bookkeeping of one env lane, packed in one register: next row to zero (bits 0-15) and the
// exclusive end of the rows that may still hold data of the slot's previous episode (bits 16-30: the slot's
// extent, T1 when unknown). Before the episode ends the next row is T1 (nothing to zero).
__device__ inline int tail_init(const MlgBatch& bt, int slot) {
    int zend = bt.T1;
    if (bt.full_write && bt.slot_extent) {
        const int x = bt.slot_extent[slot];
        zend = x < 0 ? 0 : (x < bt.T1 ? x : bt.T1);
    }
    return bt.T1 | (zend << 16);
}
__device__ inline int tail_start(int zc, int row) { return (zc & ~0xFFFF) | row; }

// Full-write (ring) mode: zero timesteps [z0, z1) of every key of batch slot `slot`.
__device__ inline void zero_slot_steps(const MlgBatch& bt, int slot, int z0, int z1, int N, int A, int S, int DO,
                                       int lane, int nl) {
    if (z0 >= z1) return;
    const int64_t r0 = (int64_t)slot * bt.T1 + z0;
    const int n = z1 - z0;  // 32-bit loop counters: fewer live VGPRs than int64 induction variables
    // obs and state rows are whole 16-byte multiples (8U and 6U floats, U even) when DO % 4 == 0 and S % 4 == 0
    auto z16 = [&](float* p, int per) {
        float* b = p + r0 * per;
        if (per % 4 == 0) {
            uint4* q = reinterpret_cast<uint4*>(b);
            for (int x = lane; x < n * per / 4; x += nl) gst(q + x, make_uint4(0u, 0u, 0u, 0u));
        } else {
            for (int x = lane; x < n * per; x += nl) gst(b + x, 0.f);
        }
    };
    z16(bt.obs, N * DO);
    z16(bt.state, S);
    int* av = bt.avail + r0 * N * A;
    float* oh = bt.actions_onehot + r0 * N * A;
    for (int x = lane; x < n * N * A; x += nl) {
        gst(av + x, 0);
        gst(oh + x, 0.f);
    }
    int64_t* ac = bt.actions + r0 * N;
    for (int x = lane; x < n * N; x += nl) gst(ac + x, (int64_t)0);
    for (int x = lane; x < n; x += nl) {
        gst(bt.reward + r0 + x, 0.f);
        gst(bt.terminated + r0 + x, (uint8_t)0);
        gst(bt.filled + r0 + x, (int64_t)0);
    }
}

// ================================================================================================
// v2 env: one half-wave (32 lanes) per env, lane u = unit u (U <= 32). Unit state lives in VGPRs for the
// whole episode; everything an env step needs from other units travels by cross-lane permutes, so the
// env phase has no workgroup barrier and no LDS round trips (same spec-v1 arithmetic as mlg_device.h,
// bit-exact; checked against v1 and the C oracle).
struct UnitMasks {
    uint32_t team1, healer, tank, melee;  // bit u set iff unit u is on plan team 1 / HEALER / TANK / MELEE
};

__device__ inline UnitMasks make_unit_masks(const SpecShared& SS, int U) {
    UnitMasks m{0u, 0u, 0u, 0u};
    for (int u = 0; u < U; ++u) {
        m.team1 |= (uint32_t)(SS.team[u] == 1) << u;
        m.healer |= (uint32_t)(SS.role[u] == 1) << u;
        m.tank |= (uint32_t)(SS.role[u] == 0) << u;
        m.melee |= (uint32_t)(SS.melee[u] == 1) << u;
    }
    return m;
}

__device__ __forceinline__ int pk_unit(int x, int y, int hp) { return x | (y << 12) | (hp << 24); }
__device__ __forceinline__ int pk_x(int q) { return q & 0xFFF; }
__device__ __forceinline__ int pk_y(int q) { return (q >> 12) & 0xFFF; }
__device__ __forceinline__ int pk_hp(int q) { return q >> 24; }
__device__ __forceinline__ int mask_role(const UnitMasks& M, int j) {
    return ((M.tank >> j) & 1) ? 0 : (((M.healer >> j) & 1) ? 1 : 2);
}
__device__ __forceinline__ int move_toward_d(int dx, int dy) {
    const int adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
    if (adx >= ady && dx != 0) return dx > 0 ? 3 : 4;
    if (dy != 0) return dy > 0 ? 1 : 2;
    return 0;
}

// Lane-resident unit of the half-wave's env.
struct UnitLane {
    int x, y, hp;        // state
    uint32_t tgt, sight; // bit j: action 5+j available / unit j visible (current state)
    int ai;              // scripted action decided on the current state (spec §3.3)
};

// One pass over all units j of the env for unit u: attack/heal availability, sight, and the scripted AI choice
// (lowest-hp target in range, else nearest ally for a healer when one is alive, else nearest enemy) -- spec
// §3.2-3.3 in mask form. U <= 16 (the latency path of every env step): the two 16-lane rows of the half-wave split
// the units j -- row 1 mirrors row 0's unit (one v_permlane16_swap), visits the upper half of j, and the partial
// masks / min-keys are combined across the rows (min and OR: exact, order-free, so the result is bit-identical to
// visiting all j in one lane).
__device__ __forceinline__ void v2_pair_pass(const UnitMasks& M, int U, int u, UnitLane& L, int* spk) {
    const uint32_t all = U >= 32 ? 0xFFFFFFFFu : ((1u << U) - 1u);
    const int hbase = (threadIdx.x & 63) & 32;
    // alive units of the env (bit j): the unit lanes of row 0 (u < U)
    const uint32_t alive_m = (uint32_t)(__ballot(u < U && L.hp > 0) >> hbase) & all;
    const int pk_own = pk_unit(L.x, L.y, L.hp);
    // packed unit states of the env through LDS (written and read by this half-wave only: in-order LDS
    // queue of one wave, no barrier)
    spk[u] = pk_own;
    const bool split = U <= 16, odd = split && (threadIdx.x & 16) != 0;
    int pkm = pk_own, uu = u;  // the unit this lane visits for: its own, or (row 1 of a split pass) row 0's
    if (split) {
        const auto sw = __builtin_amdgcn_permlane16_swap((unsigned)pk_own, (unsigned)pk_own, false, false);
        pkm = odd ? (int)sw[0] : pk_own;
        uu = u & 15;
    }
    const int X = pk_x(pkm), Y = pk_y(pkm), HP = pk_hp(pkm);
    const int my_team = (M.team1 >> uu) & 1;
    const bool healer = (M.healer >> uu) & 1;
    const int r2 = ((M.melee >> uu) & 1) ? 2 : 9;
    const bool alive = HP > 0;
    const uint32_t mates = (my_team ? M.team1 : ~M.team1) & all;
    const uint32_t cand_a = alive ? (mates & alive_m & ~(1u << uu)) : 0u;
    const uint32_t cand_e = alive ? (~mates & alive_m & all) : 0u;
    const uint32_t seen = alive ? alive_m : 0u;
    // min-keys (value << 5 | j) give "smallest value, then lowest j" -- the spec's tie rule -- without branches
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    uint32_t kbest = NONE, kally = NONE, kenemy = NONE, tgt = 0, sight = 0;
    auto visit = [&](int j, int q) {  // j may differ per lane; bits of j >= U are clear in every candidate mask
        const int hj = pk_hp(q);
        const int dx = pk_x(q) - X, dy = pk_y(q) - Y;
        const uint32_t d2 = (uint32_t)(__mul24(dx, dx) + __mul24(dy, dy));
        const uint32_t bit = 1u << j;
        const bool vis = (seen & bit) && d2 <= MLG_SIGHT2;
        const bool inr = d2 <= (uint32_t)r2;
        const int mxj = (M.tank & bit) ? 64 : 32;
        const bool tg = inr && (healer ? ((cand_a & bit) && hj < mxj) : (cand_e & bit) != 0);
        sight |= vis ? bit : 0u;
        tgt |= tg ? bit : 0u;
        kbest = min(kbest, tg ? ((uint32_t)hj << 5 | j) : NONE);
        kally = min(kally, (cand_a & bit) ? (d2 << 5 | j) : NONE);
        kenemy = min(kenemy, (cand_e & bit) ? (d2 << 5 | j) : NONE);
    };
    if (split) {
        const int JH = (U + 1) >> 1, base = odd ? JH : 0;
        int q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = k < JH ? spk[(base + k) & 31] : 0;  // all reads issued together
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (k < JH) visit((base + k) & 31, q[k]);
        auto other = [&](uint32_t v) {  // the value of lane l ^ 16
            const auto s2 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            return (threadIdx.x & 16) ? s2[0] : s2[1];
        };
        kbest = min(kbest, other(kbest));
        kally = min(kally, other(kally));
        kenemy = min(kenemy, other(kenemy));
        tgt |= other(tgt);
        sight |= other(sight);
    } else {
        for (int j0 = 0; j0 < U; j0 += 4) {  // four units per 16-byte broadcast load
            const int4 q4 = *reinterpret_cast<const int4*>(spk + j0);
            visit(j0, q4.x);
            if (j0 + 1 < U) visit(j0 + 1, q4.y);
            if (j0 + 2 < U) visit(j0 + 2, q4.z);
            if (j0 + 3 < U) visit(j0 + 3, q4.w);
        }
    }
    int ai = 0;
    if (alive) {
        uint32_t k = NONE;
        if (kbest != NONE) ai = MLG_ACT_BASE + (int)(kbest & 31);
        else if (healer && kally != NONE) k = (kally >> 5) > 2 ? kally : NONE;
        else k = kenemy;
        if (ai == 0 && k != NONE) {
            const int q = spk[k & 31];
            ai = move_toward_d(pk_x(q) - X, pk_y(q) - Y);
        }
    }
    L.tgt = tgt;  // row 1 of a split pass: lanes u >= U (no unit), whose fields no reader uses
    L.sight = sight;
    L.ai = ai;
}

// Damage and heal received by unit hl from the executed actions of all units (spec §3.4 resolution on the
// pre-step state: pk = packed pre-step units, act = executed actions, both per env in LDS). U <= 16: split across
// the two 16-lane rows (as v2_pair_pass): row 1 sums the upper half of the attackers i for row 0's unit, the
// integer partial sums are combined by one permlane16 swap each (exact).
__device__ __forceinline__ void resolve_hits(const UnitMasks& M, int U, int hl, const int* spk, const int* sact, int& dmg,
                                             int& heal) {
    if (U <= 16) {
        const bool odd = (hl & 16) != 0;
        const int me = MLG_ACT_BASE + (hl & 15), JH = (U + 1) >> 1, base = odd ? JH : 0;
        int qs[8], as[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {  // all reads issued together
            qs[k] = k < JH ? spk[(base + k) & 31] : 0;
            as[k] = k < JH ? sact[(base + k) & 31] : 0;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k >= JH) break;
            const int i = base + k;
            const bool hit = i < U && pk_hp(qs[k]) > 0 && as[k] == me;
            const bool hl_i = (M.healer >> i) & 1;
            heal += (hit && hl_i) ? role_power(1) : 0;
            dmg += (hit && !hl_i) ? role_power(mask_role(M, i)) : 0;
        }
        const auto sd = __builtin_amdgcn_permlane16_swap((unsigned)dmg, (unsigned)dmg, false, false);
        const auto sh = __builtin_amdgcn_permlane16_swap((unsigned)heal, (unsigned)heal, false, false);
        dmg += (int)(odd ? sd[0] : sd[1]);
        heal += (int)(odd ? sh[0] : sh[1]);
        return;
    }
    const int me = MLG_ACT_BASE + hl;
    for (int i0 = 0; i0 < U; i0 += 4) {  // four units per 16-byte broadcast load
        const int4 q4 = *reinterpret_cast<const int4*>(spk + i0);
        const int4 a4 = *reinterpret_cast<const int4*>(sact + i0);
        const int qs[4] = {q4.x, q4.y, q4.z, q4.w}, as[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + r;
            const bool hit = i < U && pk_hp(qs[r]) > 0 && as[r] == me;
            const bool hl_i = (M.healer >> i) & 1;
            heal += (hit && hl_i) ? role_power(1) : 0;
            dmg += (hit && !hl_i) ? role_power(mask_role(M, i)) : 0;
        }
    }
}

// Hit points lost per team over the step, summed over the half-wave's unit lanes without cross-lane permutes: one
// ballot per bit of the per-unit loss (0..64, 7 bits) and scalar popcounts by team (exact integer sums; the
// shuffle-tree reduction it replaces cost five LDS permute round trips on the env step's latency path).
__device__ __forceinline__ void team_losses(const UnitMasks& M, int loss, int hbase, int& lost0, int& lost1) {
    lost0 = lost1 = 0;
#pragma unroll
    for (int b = 0; b < 7; ++b) {
        const uint32_t m = (uint32_t)(__ballot((loss >> b) & 1) >> hbase);
        lost0 += __builtin_popcount(m & ~M.team1) << b;
        lost1 += __builtin_popcount(m & M.team1) << b;
    }
}

__device__ __forceinline__ int v2_avail(const UnitMasks& M, int G, int x, int y, int hp, uint32_t tgt, int k) {
    const bool alive = hp > 0;
    if (k == 0) return !alive;
    if (!alive) return 0;
    if (k == 1) return y + 1 < G;
    if (k == 2) return y - 1 >= 0;
    if (k == 3) return x + 1 < G;
    if (k == 4) return x - 1 >= 0;
    return (int)((tgt >> (k - MLG_ACT_BASE)) & 1u);
}

// obs / state / avail of batch index t for the half-wave's env (all 32 lanes call; `on` uniform per half).
__device__ __forceinline__ void v2_observe(const UnitMasks& M, const MlgEnvSpec& spec, const SpecShared& SS,
                                           const int* pairtab, const int* avtab, const MlgBatch& bt, int slot, int t,
                                           int e, int hbase, int hl, const UnitLane& L, float* lobs, int ldo,
                                           uint64_t* lavm, float inv_p, Stamps& sp, bool obf, int U, int N, int A,
                                           bool sd) {
    const int S = 6 * U, DO = 8 * U, G = spec.grid;
    const int64_t st_row = (int64_t)slot * bt.T1 + t;
    const int pk = pk_unit(L.x, L.y, L.hp);
#pragma unroll 1  // rolled: unrolled (static dims) it pushes the v7 kernel past 256 VGPRs
    for (int k0 = 0; k0 < N * U; k0 += 32) {
        const int k = k0 + hl;
        const bool valid = k < N * U;
        const int kk = valid ? k : 0;
        const int pt = sd ? ((kk / U) << 8) | (kk % U) : pairtab[kk];
        const int a = pt >> 8, j = pt & 255, i = SS.aunit[a];
        const int qi = __shfl(pk, hbase + i, 64), qj = __shfl(pk, hbase + j, 64);
        const uint32_t ti = __shfl((int)L.tgt, hbase + i, 64), si = __shfl((int)L.sight, hbase + i, 64);
        floatx4 lo{0.f, 0.f, 0.f, 0.f}, hi{0.f, 0.f, 0.f, 0.f};
        if ((si >> j) & 1u) {
            const int rj = mask_role(M, j);
            lo = floatx4{1.0f, (float)(pk_x(qj) - pk_x(qi)) * inv_p, (float)(pk_y(qj) - pk_y(qi)) * inv_p,
                         (float)pk_hp(qj) * inv_maxhp(rj)};
            hi = floatx4{(float)((ti >> j) & 1u), (float)(((M.team1 >> j) & 1) == ((M.team1 >> i) & 1)),
                         (float)rj * 0.5f, (float)((M.melee >> j) & 1)};
        }
        if (valid) {
            float* dst = bt.obs + (st_row * N + a) * DO + j * 8;
            gst(reinterpret_cast<floatx4*>(dst), lo);
            gst(reinterpret_cast<floatx4*>(dst + 4), hi);
            if (obf) {  // v7: bf16 rows (every obs feature is exact in bf16: k/32, hp/max_hp, 0, 0.5, 1)
                *reinterpret_cast<uint4*>(lobs + (e * N + a) * ldo + j * 4) =
                    make_uint4(cvt_pk_bf16(lo.x, lo.y), cvt_pk_bf16(lo.z, lo.w), cvt_pk_bf16(hi.x, hi.y),
                               cvt_pk_bf16(hi.z, hi.w));
            } else {
                float* l = lobs + (e * N + a) * ldo + j * 8;
                *reinterpret_cast<floatx4*>(l) = lo;
                *reinterpret_cast<floatx4*>(l + 4) = hi;
            }
        }
    }
    sp.mark(9);
    // avail: every unit lane forms its row as a bit mask (noop iff dead; moves in bounds; targets = tgt bits),
    // agent lanes publish it for the agent phase (LDS), then the half-wave writes the int rows to the batch
    {
        const bool alive = L.hp > 0;
        const uint64_t m = !alive ? 1ull
                                  : (((uint64_t)L.tgt << MLG_ACT_BASE) | ((uint64_t)(L.y + 1 < G) << 1) |
                                     ((uint64_t)(L.y - 1 >= 0) << 2) | ((uint64_t)(L.x + 1 < G) << 3) |
                                     ((uint64_t)(L.x - 1 >= 0) << 4));
        const int ag = hl < U ? SS.agent[hl] : 0;
        if (ag) lavm[e * N + ag - 1] = m;
    }
#pragma unroll 1  // rolled: see the one-hot loop in env_lane_step1
    for (int k0 = 0; k0 < N * A; k0 += 32) {
        const int k = k0 + hl;
        if (k < N * A) {
            const int pt = sd ? ((k / A) << 8) | (k % A) : avtab[k];
            gst(bt.avail + st_row * N * A + k, (int)((lavm[e * N + (pt >> 8)] >> (pt & 255)) & 1ull));
        }
    }
    sp.mark(11);
    if (hl < U) {
        const int r = mask_role(M, hl);
        float* dst = bt.state + st_row * S + hl * 6;
        gst(reinterpret_cast<float2*>(dst), make_float2((float)(L.hp > 0), (float)L.x * inv_p));
        gst(reinterpret_cast<float2*>(dst + 2), make_float2((float)L.y * inv_p, (float)L.hp * inv_maxhp(r)));
        gst(reinterpret_cast<float2*>(dst + 4), make_float2((float)((M.team1 >> hl) & 1), (float)r * 0.5f));
    }
    sp.mark(12);
}

// ================================================================================================
// v2: the headline kernel (H in {32, 64}, U <= 32; everything the step reads resident on chip).
//
// Agent phase. Work per timestep is split into (tile, 16-feature chunk) units so that all four SIMDs carry
// the same MFMA load whatever the tile count (5 tiles of 16 rows for 16 envs x 5 agents), and only rows
// of envs still running are processed: running envs are compacted into tiles every step.
//   wave w owns feature chunk j = w % HC of the GRU for tiles w / HC, w / HC + 8 / HC, ...; its
//   W_ih / W_hh rows for that chunk (3 gates x 16 features x H) live in VGPRs for the whole episode.
//   fc1 weights, fc2 weights, biases, the obs and avail rows of the current step, fc1 output x and the
//   hidden state h (double buffered, indexed by env row) live in LDS.
//   A: fc1 + ReLU per (tile, chunk) -> x        B: GRU per (tile, chunk) -> h'      C: fc2 + select per tile
// Arithmetic order is identical to v1 (same chunked K order, same bias folding).
// Env phase: half-wave per env, lane per unit (v2 env above); wave w steps envs 2w and 2w + 1.
// Barriers per step: A|B, B|C, C|env, env|A.
struct RolloutLds2 {
    int32_t w1o, w1a, w1n, b1, w2, b2, gb, obs, avail, xb, hb, hsz, pairtab, avtab, pk, act, am, rmap, hpl, total;
    int ldo, ldh, nhb;  // nhb: hidden-state buffers (2: double buffered by step parity, v2; 1: v7, see below)
    int xpl;            // v7: x held as three bf16 planes per row, row stride XPL_STRIDE words (0: fp32 rows)
    int rms;            // v7: words per wave row map
    RoEnvLds env;
};

// v7 x planes: row = 3 pieces x 64 bf16 (128 B each) + 16 B pad -> 100 words, so the 16 rows of an MFMA B read
// start on distinct bank quads (100 mod 64 = 36).
constexpr int XPL_STRIDE = 100;

__host__ __device__ constexpr RolloutLds2 make_rollout_lds2(const AgentLayout& L, int U, int N, int rew, int nhb = 2,
                                                            int xpl = 0) {
    RolloutLds2 r{};
    r.xpl = xpl;
    // v7 (xpl): obs rows and W1 obs-column rows as bf16, K padded to a multiple of 32 (Kp); row stride Kp / 2 + 4
    // words (an odd multiple of 4: the 16 rows of an MFMA operand read start on distinct bank quads); W1 held as
    // three bf16 planes (W1 = p0 + p1 + p2 exactly). Else fp32 rows of Dob + 4 floats.
    r.ldo = xpl ? ((L.Dob + 31) / 32 * 32) / 2 + 4 : L.Dob + 4;
    r.ldh = L.H + 4;
    int64_t o = 0;
    r.w1o = ro_take(o, (int64_t)(xpl ? 3 : 1) * L.H * r.ldo);
    r.w1a = ro_take(o, L.last_action ? (int64_t)L.A * r.ldh : 0);
    r.w1n = ro_take(o, L.agent_id ? (int64_t)N * r.ldh : 0);
    r.b1 = ro_take(o, L.H);
    r.w2 = ro_take(o, (int64_t)L.Ap * r.ldh);
    r.b2 = ro_take(o, L.Ap);
    r.gb = ro_take(o, 4 * L.H);
    const int rows = rew * N, rows16 = (rows + 15) / 16 * 16;
    // v7: one fp32 hidden-state buffer (updated in place: each lane reads and writes only its own two features of a
    // row, the GRU's h operand comes from the h planes below), so nhb is 1.
    if (xpl) nhb = 1;
    r.obs = ro_take(o, (int64_t)rows * r.ldo);
    r.avail = ro_take(o, (int64_t)rows * 2);  // uint64 avail mask per agent row
    r.xb = ro_take(o, (int64_t)rows16 * (xpl ? XPL_STRIDE : r.ldh));
    // v7: h' of step t as three bf16 planes per compact row of step t (split once, by the fc2 phase), the GRU's h
    // operand at step t + 1 (x-plane row layout)
    r.hpl = ro_take(o, xpl ? (int64_t)rows16 * XPL_STRIDE : 0);
    r.hsz = mlg_align4((int64_t)rows * r.ldh);
    r.nhb = nhb;
    r.hb = ro_take(o, nhb * r.hsz);
    // index tables: v7 computes them arithmetically (no LDS)
    r.pairtab = ro_take(o, xpl ? 0 : (int64_t)N * U);
    r.avtab = ro_take(o, xpl ? 0 : (int64_t)N * L.A);
    r.pk = ro_take(o, (int64_t)rew * 32);
    r.act = ro_take(o, (int64_t)rew * 32);
    r.am = ro_take(o, 16);
    r.rms = rows16 + 16;
    r.rmap = ro_take(o, 8 * r.rms);  // v7: one compact-row map per wave
    r.env = xpl ? make_env_lds_v2(o, N, rew < RE ? rew : RE) : make_env_lds(o, U, N, rew < RE ? rew : RE);
    r.total = o;
    return r;
}



__device__ __forceinline__ int nth_set_bit(uint32_t m, int k) {
    for (int i = 0; i < k; ++i) m &= m - 1;
    return __builtin_ctz(m);
}

// Workgroup-wide prologue of the v2 / v7 kernels: spec tables, small weights -> LDS (padded rows), activation
// buffers zeroed (the obs pad columns stay zero), index tables.
__device__ void v2_prologue(const MlgEnvSpec& spec, const AgentLayout& L, const float* __restrict__ P,
                            const RolloutLds2& lay, int* smem, int rows) {
    float* fm = reinterpret_cast<float*>(smem);
    SpecShared& SS = *reinterpret_cast<SpecShared*>(smem + lay.env.spec);
    const int tid = threadIdx.x, nthr = blockDim.x, H = L.H, N = spec.n_agents, U = spec.U, A = spec.n_actions;
    load_spec_tables(spec, SS);
    auto rows_cp = [&](int64_t src, int64_t dst, int nr, int nc, int ld) {
        for (int i = tid; i < nr * nc; i += nthr) fm[dst + (int64_t)(i / nc) * ld + i % nc] = P[src + i];
    };
    for (int64_t i = tid; i < (int64_t)rows * lay.ldo; i += nthr) fm[lay.obs + i] = 0.f;
    for (int64_t i = tid; i < (int64_t)lay.nhb * lay.hsz; i += nthr) fm[lay.hb + i] = 0.f;
    if (lay.xpl) {  // v7: W1 obs columns as three bf16 planes [3][H][2 ldo], zero-padded to Kp
        const int Kp = 2 * (lay.ldo - 4), pl = H * lay.ldo;
        unsigned short* w = reinterpret_cast<unsigned short*>(fm + lay.w1o);
        for (int i = tid; i < H * Kp; i += nthr) {
            const int f = i / Kp, k = i % Kp;
            float v = k < L.Dob ? P[L.w1o + (int64_t)f * L.Dob + k] : 0.f;
#pragma unroll
            for (int lvl = 0; lvl < 3; ++lvl) {
                const unsigned int pk = cvt_pk_bf16(v, 0.f);
                w[2 * (lvl * pl + f * lay.ldo) + k] = (unsigned short)(pk & 0xFFFFu);
                v -= __uint_as_float(pk << 16);
            }
        }
    } else {
        rows_cp(L.w1o, lay.w1o, H, L.Dob, lay.ldo);
    }
    if (L.last_action) rows_cp(L.w1a, lay.w1a, L.A, H, lay.ldh);
    if (L.agent_id) rows_cp(L.w1n, lay.w1n, N, H, lay.ldh);
    rows_cp(L.b1, lay.b1, 1, H, H);
    rows_cp(L.w2, lay.w2, L.Ap, H, lay.ldh);
    rows_cp(L.b2, lay.b2, 1, L.Ap, L.Ap);
    rows_cp(L.brz, lay.gb, 1, 2 * H, 2 * H);
    rows_cp(L.bih + 2 * H, lay.gb + 2 * H, 1, H, H);
    rows_cp(L.bhh + 2 * H, lay.gb + 3 * H, 1, H, H);
    if (!lay.xpl) {
        for (int k = tid; k < N * U; k += nthr) smem[lay.pairtab + k] = ((k / U) << 8) | (k % U);
        for (int k = tid; k < N * A; k += nthr) smem[lay.avtab + k] = ((k / A) << 8) | (k % A);
    } else {  // v7: h planes of step -1 = 0 (h_0 = 0)
        for (int64_t i = tid; i < (int64_t)(rows + 15) / 16 * 16 * XPL_STRIDE; i += nthr) fm[lay.hpl + i] = 0.f;
    }
    __syncthreads();
}

// ---- agent phase pieces (v2) ---------------------------------------------------------------------
// The wave's GRU weight rows for feature chunk j (3 gates x 16 features x H, A-operand layout) + biases.
template <int H>
struct GruChunk {
    floatx4 wi[3][H / 16], wh[3][H / 16];
    int gbo;  // LDS float index of the chunk's gate biases (r, z, ih_n, hh_n at +0, +H, +2H, +3H): read per
              // unit instead of held in 16 VGPRs (the step loop is at the 256-VGPR limit)
};

template <int H>
__device__ inline void load_gru_chunk(GruChunk<H>& W, const float* __restrict__ P, const AgentLayout& L, const float* fm,
                                      const RolloutLds2& lay, int j, int lane) {
    constexpr int HC = H / 16;
    const int col = lane & 15, g = lane >> 4;
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int kc = 0; kc < HC; ++kc) {
            const int64_t r = (int64_t)(q * H + j * 16 + col) * H + kc * 16 + 4 * g;
            W.wi[q][kc] = ld4(P + L.wih + r);
            W.wh[q][kc] = ld4(P + L.whh + r);
        }
    W.gbo = lay.gb + j * 16 + 4 * g;
    // Consume the loaded registers here, before the episode loop: the empty asm "reads" them, so the compiler's
    // waitcnt for these loads lands outside the loop. Otherwise its loop-header merge keeps them pending and
    // re-issues vmcnt waits at their first use inside the loop on every step -- which, vmcnt being in order,
    // also waits for the previous step's batch stores.
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int kc = 0; kc < HC; ++kc) asm volatile("" : "+v"(W.wi[q][kc]), "+v"(W.wh[q][kc]));
}

// Compacted agent rows of one step: the living agents of the running envs ebase .. ebase + ne - 1 (amask[e]
// bit n = agent n of env e needs a Q this step; dead agents' actions are forced to no-op by the spec, so their
// cell is skipped and the env phase records the no-op). Row cr -> env of the first inclusive prefix P[l] > cr,
// agent = (cr - P[l - 1])-th set bit of its mask. P is wave-uniform (readlane of a 16-lane scan).
struct StepRows {
    int P[16];
    const uint32_t* amask;
    int ebase, rows_run, tiles;
    __device__ bool at(int cr, int& e, int& n) const {
        const bool v = cr < rows_run;
        const int c = v ? cr : 0;
        int k = 0, base = 0;
#pragma unroll
        for (int l = 0; l < 16; ++l) {
            const bool le = P[l] <= c;
            k += le;
            base = le ? P[l] : base;
        }
        e = ebase + k;
        n = nth_set_bit(amask[e], c - base);
        return v;
    }
};

__device__ inline StepRows make_rows(const uint32_t* amask, int ebase, int ne, int lane) {
    StepRows s;
    s.amask = amask;
    s.ebase = ebase;
    const int l16 = lane & 15;
    int c = group_incl_scan<16>(l16 < ne ? __builtin_popcount(amask[ebase + l16]) : 0, lane);
#pragma unroll
    for (int l = 0; l < 16; ++l) s.P[l] = __builtin_amdgcn_readlane(c, l);
    s.rows_run = s.P[15];
    s.tiles = (s.rows_run + 15) / 16;
    return s;
}

// A: fc1 + ReLU for (tile, chunk j) over tiles ti0, ti0 + dt, ...  -> x (compact rows)

template <int H>
__device__ inline void ph_fc1(const AgentLayout& L, const RolloutLds2& lay, float* fm, const int* prev,
                              const StepRows& SR, int j, int ti0, int dt, int t, int lane) {
    const int col = lane & 15, g = lane >> 4, N = L.N, ldo = lay.ldo, ldh = lay.ldh, KO = L.Dob / 16;
    const float* lobs = fm + lay.obs;
    for (int ti = ti0; ti < SR.tiles; ti += dt) {
        int zero = 0;
        asm volatile("" : "+s"(zero));
        const int cr = ti * 16 + col;
        int e, n;
        const bool valid = SR.at(cr, e, n);
        const int er = e * N + n;
        floatx4 acc = ld4(fm + lay.b1 + zero + j * 16 + 4 * g);
        const int pa = (valid && t > 0) ? prev[er] : -1;
        if (L.last_action && pa >= 0) acc += ld4(fm + lay.w1a + (int64_t)pa * ldh + j * 16 + 4 * g);
        if (L.agent_id) acc += ld4(fm + lay.w1n + (int64_t)n * ldh + j * 16 + 4 * g);
        const float* orow = lobs + (int64_t)er * ldo + 4 * g;
        const float* wrow = fm + lay.w1o + zero + (int64_t)(j * 16 + col) * ldo + 4 * g;
        for (int kc = 0; kc < KO; ++kc) acc = mfma_chunk(ld4(wrow + kc * 16), ld4(orow + kc * 16), acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = fmaxf(acc[r], 0.f);
        *reinterpret_cast<floatx4*>(fm + lay.xb + (int64_t)cr * ldh + j * 16 + 4 * g) = acc;
    }
}

// B: GRU cell for (tile, chunk j) -> h' (rows of running envs, hidden state indexed by env row).
template <int H>
__device__ inline void ph_gru(const GruChunk<H>& W, const RolloutLds2& lay, float* fm, const float* hc, float* hn,
                              const StepRows& SR, int N_, int j, int ti0, int dt, int lane) {
    constexpr int HC = H / 16;
    const int col = lane & 15, g = lane >> 4, N = N_, ldh = lay.ldh;
    for (int ti = ti0; ti < SR.tiles; ti += dt) {
        const int cr = ti * 16 + col;
        int e, n;
        const bool valid = SR.at(cr, e, n);
        const int er = e * N + n;
        const float* xr = fm + lay.xb + (int64_t)cr * ldh + 4 * g;
        const float* hr = hc + (int64_t)er * ldh + 4 * g;
        const float* gbp = fm + W.gbo;
        floatx4 ar = ld4(gbp), az = ld4(gbp + H), ain = ld4(gbp + 2 * H), ahn = ld4(gbp + 3 * H);
#pragma unroll
        for (int kc = 0; kc < HC; ++kc) {
            const floatx4 xin = ld4(xr + kc * 16), hin = ld4(hr + kc * 16);
            ar = mfma_chunk(W.wi[0][kc], xin, ar);
            az = mfma_chunk(W.wi[1][kc], xin, az);
            ain = mfma_chunk(W.wi[2][kc], xin, ain);
            ar = mfma_chunk(W.wh[0][kc], hin, ar);
            az = mfma_chunk(W.wh[1][kc], hin, az);
            ahn = mfma_chunk(W.wh[2][kc], hin, ahn);
        }
        const floatx4 ho = ld4(hr + j * 16);
        floatx4 hv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float rg = 1.f / (1.f + expf(-ar[r]));
            const float zg = 1.f / (1.f + expf(-az[r]));
            const float ng = tanhf(ain[r] + rg * ahn[r]);
            hv[r] = ng + zg * (ho[r] - ng);
        }
        if (valid) *reinterpret_cast<floatx4*>(hn + (int64_t)er * ldh + j * 16 + 4 * g) = hv;
    }
}

// ---- v7 row map -------------------------------------------------------------------------------------------
// Compacted agent rows of the step (as StepRows) as an LDS table private to the wave: entry cr = env e << 8 |
// agent n << 1 | 1 (0 for tile padding). Lanes 0-15 (one per env) scatter their env's living agents after a
// 16-lane scan of the agent counts; the wave reads its own table back (LDS is in order within a wave), so no
// workgroup barrier and no SGPR-resident prefix array. Returns the tile count.
// Row-map entry: bit 0 valid, bits 1-7 agent n, bits 8-15 env e, bits 16-23 (v7) the row's compact index at the
// previous step (where its h' planes are, HPL).
__device__ __forceinline__ int rmap_env(int rm) { return (rm >> 8) & 255; }
__device__ __forceinline__ int rmap_er(int rm, int N) { return rmap_env(rm) * N + ((rm >> 1) & 127); }
__device__ __forceinline__ int rmap_prev(int rm) { return (rm >> 16) & 255; }

// m: amask[lane & 15]; m_prev / x_prev (lanes 0-15): the env's agent mask and exclusive row prefix of the previous
// step (0 / 0 before the first: row 0 of the zeroed h planes), updated here. Rows only disappear between steps
// (agents die, envs end), so a row's previous compact index is x_prev + the number of its env's earlier agents
// in m_prev.
__device__ inline int make_rmap(uint32_t m, int* wmap, int lane, uint32_t& m_prev, int& x_prev) {
    int c = group_incl_scan<16>(__builtin_popcount(m), lane);
    const int rows = __builtin_amdgcn_readlane(c, 15);
    const int x = c - __builtin_popcount(m);
    if (lane < 16) {
        int p = x;
        for (uint32_t mm = m; mm; mm &= mm - 1) {
            const int n = __builtin_ctz(mm);
            const int cp = x_prev + __builtin_popcount(m_prev & ((1u << n) - 1u));
            wmap[p++] = (cp << 16) | (lane << 8) | (n << 1) | 1;
        }
        wmap[rows + lane] = 0;  // padding rows of the last tile
    }
    m_prev = m;
    x_prev = x;
    return (rows + 15) >> 4;
}

// v7 A: fc1 + ReLU for (tile, chunk j) as ph_fc1 (same fp32 arithmetic), rows from the wave's row map, x stored
// as three bf16 planes (x = p0 + p1 + p2 exactly) = the GRU's B operands, split once here.
template <int H>
__device__ inline void ph_fc1_g8(const AgentLayout& L, const RolloutLds2& lay, float* fm, const int* rmap, const int* prev,
                                 int tiles, int j, int ti0, int dt, int t, int lane) {
    const int col = lane & 15, g = lane >> 4, N = L.N, ldo = lay.ldo, ldh = lay.ldh, KK = (L.Dob + 31) / 32;
    const float* lobs = fm + lay.obs;
    for (int ti = ti0; ti < tiles; ti += dt) {
        int zero = 0;
        asm volatile("" : "+s"(zero));
        const int cr = ti * 16 + col;
        const int rm = rmap[cr];
        const bool valid = rm & 1;
        const int n = (rm >> 1) & 127, er = rmap_er(rm, N);
        floatx4 acc = ld4(fm + lay.b1 + zero + j * 16 + 4 * g);
        const int pa = (valid && t > 0) ? prev[er] : -1;
        if (L.last_action && pa >= 0) acc += ld4(fm + lay.w1a + pa * ldh + j * 16 + 4 * g);
        if (L.agent_id) acc += ld4(fm + lay.w1n + n * ldh + j * 16 + 4 * g);
        // bf16 obs row (exact) x W1 as three bf16 planes: 3 partial products per 32-wide K step, all exact, fp32
        // accumulation (the same fp32-class arithmetic as the GRU, §4a)
        const bf16x8* orow = reinterpret_cast<const bf16x8*>(lobs + er * ldo) + g;
        const bf16x8* wrow = reinterpret_cast<const bf16x8*>(fm + lay.w1o + zero + (j * 16 + col) * ldo) + g;
        const int pl = L.H * ldo / 4;  // plane stride in bf16x8 units
        for (int kk = 0; kk < KK; ++kk) {
            const bf16x8 b = orow[4 * kk];
            acc = mfma_bf16(wrow[2 * pl + 4 * kk], b, acc);
            acc = mfma_bf16(wrow[pl + 4 * kk], b, acc);
            acc = mfma_bf16(wrow[4 * kk], b, acc);
        }
        unsigned int* xr = reinterpret_cast<unsigned int*>(fm + lay.xb + cr * XPL_STRIDE) + (j * 16 + 4 * g) / 2;
        float v[4] = {fmaxf(acc[0], 0.f), fmaxf(acc[1], 0.f), fmaxf(acc[2], 0.f), fmaxf(acc[3], 0.f)};
#pragma unroll
        for (int lvl = 0; lvl < 3; ++lvl) {
            const unsigned int a = cvt_pk_bf16(v[0], v[1]), b = cvt_pk_bf16(v[2], v[3]);
            *reinterpret_cast<uint2*>(xr + lvl * 32) = make_uint2(a, b);
            if (lvl < 2) {
                v[0] -= __uint_as_float(a << 16);
                v[1] -= __uint_as_float(a & 0xFFFF0000u);
                v[2] -= __uint_as_float(b << 16);
                v[3] -= __uint_as_float(b & 0xFFFF0000u);
            }
        }
    }
}

// v7 A for the static plan shapes: the wave's NU (tile, chunk j) units of ph_fc1_g8 as one straight-line block
// (identical arithmetic per unit). ph_fc1_g8 walks its units one after another, each a chain of dependent LDS
// round trips (row map -> previous action -> last-action column) feeding a 9-deep MFMA chain, then the split and
// the x-plane stores: at full occupancy (3 units per wave) fc1 took 4.7 k cycles per step against ~0.4 k of
// MFMA work. Here every LDS read of all units issues first, the chunk's W1 operands are read once (they do not
// depend on the tile), and the units' MFMA chains interleave.
template <int H, int KK, int NU>
__device__ __forceinline__ void fc1_g8_units(const AgentLayout& L, const RolloutLds2& lay, float* fm, const int* rmap,
                                             const int* prev, int j, int ti0, int dt, int t, int lane) {
    const int col = lane & 15, g = lane >> 4, N = L.N, ldo = lay.ldo, ldh = lay.ldh;
    int zero = 0;
    asm volatile("" : "+s"(zero));
    const float* lobs = fm + lay.obs;
    int cr[NU], er[NU], n[NU];
    bool valid[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        cr[u] = (ti0 + u * dt) * 16 + col;
        const int rm = rmap[cr[u]];
        valid[u] = rm & 1;
        n[u] = (rm >> 1) & 127;
        er[u] = rmap_er(rm, N);
    }
    const bf16x8* orow[NU];
    int pa[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        orow[u] = reinterpret_cast<const bf16x8*>(lobs + er[u] * ldo) + g;
        pa[u] = (valid[u] && t > 0) ? prev[er[u]] : -1;
    }
    const bf16x8* wrow = reinterpret_cast<const bf16x8*>(fm + lay.w1o + zero + (j * 16 + col) * ldo) + g;
    const int pl = L.H * ldo / 4;  // plane stride in bf16x8 units
    const floatx4 b1 = ld4(fm + lay.b1 + zero + j * 16 + 4 * g);
    floatx4 acc[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        acc[u] = b1;
        if (L.last_action && pa[u] >= 0) acc[u] += ld4(fm + lay.w1a + pa[u] * ldh + j * 16 + 4 * g);
        if (L.agent_id) acc[u] += ld4(fm + lay.w1n + n[u] * ldh + j * 16 + 4 * g);
    }
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {  // operands per K step (register budget: the kernel runs at 2 waves / SIMD)
        bf16x8 w[3], b[NU];
#pragma unroll
        for (int p = 0; p < 3; ++p) w[p] = wrow[p * pl + 4 * kk];
#pragma unroll
        for (int u = 0; u < NU; ++u) b[u] = orow[u][4 * kk];
#pragma unroll
        for (int p = 2; p >= 0; --p)
#pragma unroll
            for (int u = 0; u < NU; ++u) acc[u] = mfma_bf16(w[p], b[u], acc[u]);
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        unsigned int* xr = reinterpret_cast<unsigned int*>(fm + lay.xb + cr[u] * XPL_STRIDE) + (j * 16 + 4 * g) / 2;
        float v[4] = {fmaxf(acc[u][0], 0.f), fmaxf(acc[u][1], 0.f), fmaxf(acc[u][2], 0.f), fmaxf(acc[u][3], 0.f)};
#pragma unroll
        for (int lvl = 0; lvl < 3; ++lvl) {
            const unsigned int a = cvt_pk_bf16(v[0], v[1]), c = cvt_pk_bf16(v[2], v[3]);
            *reinterpret_cast<uint2*>(xr + lvl * 32) = make_uint2(a, c);
            if (lvl < 2) {
                v[0] -= __uint_as_float(a << 16);
                v[1] -= __uint_as_float(a & 0xFFFF0000u);
                v[2] -= __uint_as_float(c << 16);
                v[3] -= __uint_as_float(c & 0xFFFF0000u);
            }
        }
    }
}

// nu (wave-uniform, 0..MU) units of fc1_g8_units: tiles ti0, ti0 + dt, ...
template <int H, int KK, int MU>
__device__ __forceinline__ void fc1_g8_static(const AgentLayout& L, const RolloutLds2& lay, float* fm, const int* rmap,
                                              const int* prev, int nu, int j, int ti0, int dt, int t, int lane) {
    if (nu == MU)
        fc1_g8_units<H, KK, MU>(L, lay, fm, rmap, prev, j, ti0, dt, t, lane);
    else if constexpr (MU > 1)
        fc1_g8_static<H, KK, MU - 1>(L, lay, fm, rmap, prev, nu, j, ti0, dt, t, lane);
}

// ---- v7 GRU: fp32 products emulated on the bf16 matrix cores (split-bf16 "bf16x6") -------------------------
// Every fp32 operand a is split into three bf16 pieces a = a0 + a1 + a2 (round to nearest each; the sum is
// exact: a0 holds the top 8 significant bits, a1 the next 8, a2 the rest, which fits a bf16), and a product
// a*b is summed as the six partial products with i + j <= 2 (a0b0, a0b1, a1b0, a0b2, a1b1, a2b0) in fp32 MFMA
// accumulators. The three dropped terms are below 2^-24 of |a b| (a1b2, a2b1: ~2^-26; a2b2: ~2^-34), so each
// product carries fp32-class error, from fp32 operands, in 6 x 16 = 96 matrix-core cycles per 16x16x32 step
// instead of 8 x 32 = 256 for v_mfma_f32_16x16x4_f32 (MI355X_MICROARCH.md cycle table). Accumulation is fp32
// inside the MFMA, in a different order than the v1/v2 fmaf chains: v7 results equal v2's to fp32 rounding,
// not bit for bit.

// Wave w owns hidden features 8w .. 8w+7 (H = 64, 8 waves): three 16-row A blocks per 32-wide K step,
//   rz_i = [W_ir ; W_iz] (rows 0-7 r, 8-15 z of its features)   with B = x
//   rz_h = [W_hr ; W_hz]                                         with B = h   (same accumulator rows)
//   n    = [W_in ; W_hn]  with B = x (rows 0-7 used) and with B = h (rows 8-15 used)
// so each weight is held once in the workgroup (72 VGPRs of bf16 pieces, v2: 96 VGPRs of fp32, every chunk
// twice). Gate pre-activations of one (feature, agent row) end up split over lanes l and l + 32; one
// permlane32_swap per register pair gives each lane two complete features.
struct GruG8 {
    Split3 rzi[2], rzh[2], n[2];
    int rz_bias, in_bias, hn_bias;  // LDS float indices of this lane's 4 bias rows
};

__device__ inline void load_gru_g8(GruG8& W, const float* __restrict__ P, const AgentLayout& L, const RolloutLds2& lay,
                                   int w, int lane) {
    const int H = L.H, row = lane & 15, g = lane >> 4, f = 8 * w + (row & 7), hi = row >> 3;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        const int k = 32 * kk + 8 * g;
        const float* ri = P + L.wih + (int64_t)(hi * H + f) * H + k;        // r (hi = 0) / z (hi = 1) row of W_ih
        const float* rh = P + L.whh + (int64_t)(hi * H + f) * H + k;
        const float* rn = P + (hi ? L.whh : L.wih) + (int64_t)(2 * H + f) * H + k;  // W_in (rows 0-7) / W_hn (8-15)
        W.rzi[kk] = split3(ld4(ri), ld4(ri + 4));
        W.rzh[kk] = split3(ld4(rh), ld4(rh + 4));
        W.n[kk] = split3(ld4(rn), ld4(rn + 4));
    }
    // accumulator rows 4g .. 4g+3: g = 0, 1 -> r / W_in of features 8w + 4g ..; g = 2, 3 -> z / W_hn of 8w + 4(g-2) ..
    const int fo = 8 * w + 4 * (g & 1);
    W.rz_bias = lay.gb + (g < 2 ? fo : H + fo);
    W.in_bias = lay.gb + 2 * H + fo;
    W.hn_bias = lay.gb + 3 * H + fo;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int q = 0; q < 3; ++q)
            asm volatile("" : "+v"(W.rzi[kk].p[q]), "+v"(W.rzh[kk].p[q]), "+v"(W.n[kk].p[q]));
}

// B: GRU cell of every tile for the wave's 8 features -> h' (env-row hidden state). x comes as bf16 planes from
// fc1 (split once), h is split here; the compact-row -> env-row map was stored by fc1.
// NT (1 or 2) consecutive tiles of ph_gru_g8 with their MFMA chains interleaved (8 independent accumulators for
// two tiles): one tile's operand loads and gate epilogue overlap the other's matrix work. Per tile the same
// operations in the same order as the one-tile loop.
template <int NT>
__device__ __forceinline__ void gru_g8_tiles(const GruG8& W, const RolloutLds2& lay, float* fm, const int* rmap, float* hb,
                                             int ti0, int N, int fo, int lane) {
    const int col = lane & 15, g = lane >> 4, ldh = lay.ldh;
    const bool upper = lane >= 32;
    int er[NT];
    bool valid[NT];
    const bf16x8 *xp[NT], *hp[NT];
    floatx4 arz[NT], arzh[NT], anx[NT], anh[NT];
#pragma unroll
    for (int u = 0; u < NT; ++u) {
        const int cr = (ti0 + u) * 16 + col;
        const int rm = rmap[cr];
        valid[u] = rm & 1;
        er[u] = rmap_er(rm, N);
        xp[u] = reinterpret_cast<const bf16x8*>(fm + lay.xb + (int64_t)cr * XPL_STRIDE) + g;
        // h of the previous step, split once per step (hpl_split_tile; HPL row = the row's previous compact index)
        hp[u] = reinterpret_cast<const bf16x8*>(fm + lay.hpl + (int64_t)rmap_prev(rm) * XPL_STRIDE) + g;
        arz[u] = ld4(fm + W.rz_bias);
        arzh[u] = floatx4{0.f, 0.f, 0.f, 0.f};
        anx[u] = ld4(fm + W.in_bias);
        anh[u] = ld4(fm + W.hn_bias);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        Split3 xs[NT], hs[NT];
#pragma unroll
        for (int u = 0; u < NT; ++u)
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                xs[u].p[p] = xp[u][p * 8 + 4 * kk];  // plane p: +128 B; K step kk: +64 B
                hs[u].p[p] = hp[u][p * 8 + 4 * kk];
            }
#pragma unroll
        for (int u = 0; u < NT; ++u) {
            arz[u] = mfma_x6(W.rzi[kk], xs[u], arz[u]);
            anx[u] = mfma_x6(W.n[kk], xs[u], anx[u]);
            arzh[u] = mfma_x6(W.rzh[kk], hs[u], arzh[u]);
            anh[u] = mfma_x6(W.n[kk], hs[u], anh[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < NT; ++u) {
        const floatx4 az = arz[u] + arzh[u];
        // lanes l < 32 hold r (rows 4g..) and W_in x; lanes l + 32 hold z and W_hn h of the same features
        float r0, r1, z0, z1;
        {
            auto s0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(az[0]), __float_as_uint(az[2]), false, false);
            auto s1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(az[1]), __float_as_uint(az[3]), false, false);
            r0 = __uint_as_float(s0[0]);
            z0 = __uint_as_float(s0[1]);
            r1 = __uint_as_float(s1[0]);
            z1 = __uint_as_float(s1[1]);
        }
        float ni0, ni1, nh0, nh1;
        {
            auto s0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(anh[u][0]), __float_as_uint(anx[u][2]), false, false);
            auto s1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(anh[u][1]), __float_as_uint(anx[u][3]), false, false);
            // lower: own anx[0..1] = W_in x, received (in the anx[2..3] slot) W_hn h; upper: received W_in x in the
            // anh[0..1] slot, own anh[2..3] = W_hn h
            ni0 = upper ? __uint_as_float(s0[0]) : anx[u][0];
            ni1 = upper ? __uint_as_float(s1[0]) : anx[u][1];
            nh0 = upper ? anh[u][2] : __uint_as_float(s0[1]);
            nh1 = upper ? anh[u][3] : __uint_as_float(s1[1]);
        }
        const float2 ho = *reinterpret_cast<const float2*>(hb + (int64_t)er[u] * ldh + fo);
        float2 hv;
        {
            const float rg = fast_sigmoid(r0), zg = fast_sigmoid(z0);
            const float ng = fast_tanh(ni0 + rg * nh0);
            hv.x = ng + zg * (ho.x - ng);
        }
        {
            const float rg = fast_sigmoid(r1), zg = fast_sigmoid(z1);
            const float ng = fast_tanh(ni1 + rg * nh1);
            hv.y = ng + zg * (ho.y - ng);
        }
        if (valid[u]) *reinterpret_cast<float2*>(hb + (int64_t)er[u] * ldh + fo) = hv;  // in place: own features only
    }
}

template <int H>
__device__ inline void ph_gru_g8(const GruG8& W, const RolloutLds2& lay, float* fm, const int* rmap, float* hb,
                                 int tiles, int N, int w, int lane) {
    // this lane's two output features after the exchange: lower lanes 8w+4g+{0,1}, upper 8w+4(g-2)+2+{0,1}
    const int fo = 8 * w + 4 * ((lane >> 4) & 1) + (lane >= 32 ? 2 : 0);
    int ti = 0;
    for (; ti + 1 < tiles; ti += 2) gru_g8_tiles<2>(W, lay, fm, rmap, hb, ti, N, fo, lane);
    for (; ti < tiles; ++ti) gru_g8_tiles<1>(W, lay, fm, rmap, hb, ti, N, fo, lane);
}

// C: fc2 + masked argmax + epsilon-greedy per tile; records the actions (batch + LDS pending actions).
template <int H>
__device__ inline void ph_fc2(const MlgEnvSpec& spec, const AgentLayout& L, const RolloutLds2& lay, float* fm,
                              const RoEnv& R, const MlgBatch& bt, const float* hn, const StepRows& SR, int ti0, int dt,
                              int e0, int t, float eps, int test_mode, int lane) {
    constexpr int HC = H / 16;
    const int col = lane & 15, g = lane >> 4, N = L.N, ldh = lay.ldh, A = spec.n_actions, n_at = L.Ap / 16;
    const uint64_t* lavm = reinterpret_cast<const uint64_t*>(fm + lay.avail);
    for (int ti = ti0; ti < SR.tiles; ti += dt) {
        int zero = 0;
        asm volatile("" : "+s"(zero));
        const int cr = ti * 16 + col;
        int e, n;
        const bool valid = SR.at(cr, e, n);
        const int er = e * N + n;
        const float* hr = hn + (int64_t)er * ldh + 4 * g;
        const uint64_t avm = lavm[er];
        ArgmaxState as{-INFINITY, 1 << 30};
        for (int at = 0; at < n_at; ++at) {
            floatx4 q = ld4(fm + lay.b2 + zero + at * 16 + 4 * g);
            const float* w2r = fm + lay.w2 + zero + (int64_t)(at * 16 + col) * ldh + 4 * g;
#pragma unroll
            for (int kc = 0; kc < HC; ++kc) q = mfma_chunk(ld4(w2r + kc * 16), ld4(hr + kc * 16), q);
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // masked argmax (argmax_accumulate on the bit mask)
                const int a = at * 16 + 4 * g + r;
                if (a >= A) continue;
                const float v = ((avm >> a) & 1ull) ? q[r] : -INFINITY;
                if (amax_better(v, a, as.bv, as.bi)) { as.bv = v; as.bi = a; }
            }
        }
        int act = argmax_reduce(as);
        if (valid && g == 0) {
            if (!test_mode && eps > 0.f) {  // epsilon-greedy (action_selectors.py:44-62), counter RNG of spec §3.7
                const uint64_t key = mlg_env_key(spec.seed, e0 + e);
                const uint64_t r1 = mlg_rng(key, mlg_ctr(R.episode[e], (uint32_t)t, MLG_PURPOSE_EPS, (uint32_t)n));
                if (mlg_u01(r1) < eps) {
                    const uint64_t r2 = mlg_rng(key, mlg_ctr(R.episode[e], (uint32_t)t, MLG_PURPOSE_RAND, (uint32_t)n));
                    const int na = __popcll(avm);  // random_available on the mask: k-th available action
                    if (na == 0) {
                        act = 0;
                    } else {
                        const int k = (int)(((r2 >> 40) * (uint64_t)na) >> 24);
                        uint64_t m = avm;
                        for (int i = 0; i < k; ++i) m &= m - 1;
                        act = __ffsll((long long)m) - 1;
                    }
                }
            }
            R.pact[e * N + n] = act;
            const int64_t bt_off = ((int64_t)R.slot[e] * bt.T1 + t) * N + n;
            gst(bt.actions + bt_off, (int64_t)act);
            if (!bt.full_write) gst(bt.actions_onehot + bt_off * A + act, 1.0f);
        }
    }
}

// Epsilon coin of this lane's row of compact tile ti (action_selectors.py:56, spec §3.7 counter RNG; the agent index
// field of the row-map entry: agent within the env, or the global agent index in the self-play map), drawn ahead of
// the fc2 phase.
__device__ __forceinline__ int eps_coin(const MlgEnvSpec& spec, const RoEnv& R, const int* rmap, int ti, int e0, int t,
                                        float eps, int test_mode, int lane) {
    const int rm = rmap[ti * 16 + (lane & 15)];
    const int e = rmap_env(rm), n = (rm >> 1) & 127;
    const uint64_t key = mlg_env_key(spec.seed, e0 + e);
    return !test_mode && eps > 0.f &&
           mlg_u01(mlg_rng(key, mlg_ctr(R.episode[e], (uint32_t)t, MLG_PURPOSE_EPS, (uint32_t)n))) < eps;
}

// v7 C: fc2 + masked argmax + epsilon-greedy per tile, rows from the fc1 row map. The epsilon draws do not depend
// on Q, so they are made before the fc2 chain (their latency overlaps the MFMAs), and fc2 accumulates the four
// 16-wide K chunks in separate chains (fp32-class like the rest of v7; same selection rule as ph_fc2).
template <int H>
__device__ inline void ph_fc2_g8(const MlgEnvSpec& spec, const AgentLayout& L, const RolloutLds2& lay, float* fm,
                                 const int* rmap, const RoEnv& R, const MlgBatch& bt, const float* hn, int tiles, int ti0,
                                 int dt, int e0, int t, float eps, int test_mode, int lane, int pre = -1) {
    constexpr int HC = H / 16;
    const int col = lane & 15, g = lane >> 4, N = L.N, ldh = lay.ldh, A = spec.n_actions, n_at = L.Ap / 16;
    const uint64_t* lavm = reinterpret_cast<const uint64_t*>(fm + lay.avail);
    for (int ti = ti0; ti < tiles; ti += dt) {
        int zero = 0;
        asm volatile("" : "+s"(zero));
        const int cr = ti * 16 + col;
        const int rm = rmap[cr];
        const bool valid = rm & 1;
        const int e = rmap_env(rm), n = (rm >> 1) & 127, er = e * N + n;
        const uint64_t avm = lavm[er];
        const float* hr = hn + er * ldh + 4 * g;
        ArgmaxState as{-INFINITY, 1 << 30};
        // epsilon-greedy coin (action_selectors.py:44-62, counter RNG of spec §3.7): computed by every lane with no
        // branch, so it issues between the fc2 MFMAs; only the rare exploring lanes take the branch below
        const uint64_t key = mlg_env_key(spec.seed, e0 + e);
        const uint32_t ep = R.episode[e];
        bool explore;  // the wave's first tile: coin drawn during the GRU phase (eps_coin), off this phase's path
        if (ti == ti0 && pre >= 0)
            explore = pre;
        else
            explore = !test_mode && eps > 0.f &&
                      mlg_u01(mlg_rng(key, mlg_ctr(ep, (uint32_t)t, MLG_PURPOSE_EPS, (uint32_t)n))) < eps;
        auto q_block = [&](int at) {  // Q rows at*16 .. at*16+15 of this lane's agent row; all operands loaded first
            const float* w2r = fm + lay.w2 + zero + (at * 16 + col) * ldh + 4 * g;
            floatx4 wk[HC], hk[HC], qk[HC];
#pragma unroll
            for (int kc = 0; kc < HC; ++kc) {
                wk[kc] = ld4(w2r + kc * 16);
                hk[kc] = ld4(hr + kc * 16);
            }
            const floatx4 b = ld4(fm + lay.b2 + zero + at * 16 + 4 * g);
#pragma unroll
            for (int kc = 0; kc < HC; ++kc) qk[kc] = mfma_chunk(wk[kc], hk[kc], floatx4{0.f, 0.f, 0.f, 0.f});
            floatx4 q = b;
#pragma unroll
            for (int kc = 0; kc < HC; ++kc) q += qk[kc];
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // masked argmax (argmax_accumulate on the bit mask), branch-free
                const int a = at * 16 + 4 * g + r;
                const float v = (a < A && ((avm >> a) & 1ull)) ? q[r] : -INFINITY;
                const bool take = a < A && amax_better(v, a, as.bv, as.bi);
                as.bv = take ? v : as.bv;
                as.bi = take ? a : as.bi;
            }
        };
        if (n_at == 1)
            q_block(0);
        else
            for (int at = 0; at < n_at; ++at) q_block(at);
        int ract = -1;  // random available action of an exploring agent
        if (explore && valid && g == 0) {
            const uint64_t r2 = mlg_rng(key, mlg_ctr(ep, (uint32_t)t, MLG_PURPOSE_RAND, (uint32_t)n));
            const int na = __popcll(avm);  // random_available on the mask: k-th available action
            ract = 0;
            if (na > 0) {
                const int k = (int)(((r2 >> 40) * (uint64_t)na) >> 24);
                uint64_t m = avm;
                for (int i = 0; i < k; ++i) m &= m - 1;
                ract = __ffsll((long long)m) - 1;
            }
        }
        int act = argmax_reduce(as);
        if (valid && g == 0) {
            if (ract >= 0) act = ract;
            R.pact[e * N + n] = act;
            const int64_t bt_off = ((int64_t)R.slot[e] * bt.T1 + t) * N + n;
            gst(bt.actions + bt_off, (int64_t)act);
            if (!bt.full_write) gst(bt.actions_onehot + bt_off * A + act, 1.0f);
        }
    }
}

// v7: h' of compact tile ti as three bf16 planes (split3's pieces: round to nearest, exact remainders) at its compact
// rows (HPL), the GRU's h operand of the next step. Run between barrier C and the end of the step (HPL is read by the
// next step's GRU after two more barriers; the fp32 h' it reads was written before barrier B).
template <int H>
__device__ inline void hpl_split_tile(const RolloutLds2& lay, float* fm, const int* rmap, const float* hb, int ti, int N,
                                      int lane) {
    constexpr int HC = H / 16;
    const int col = lane & 15, g = lane >> 4, cr = ti * 16 + col, rm = rmap[cr];
    if (!(rm & 1)) return;
    const float* hr = hb + rmap_er(rm, N) * lay.ldh + 4 * g;
    unsigned int* hq = reinterpret_cast<unsigned int*>(fm + lay.hpl + cr * XPL_STRIDE) + 2 * g;
#pragma unroll
    for (int kc = 0; kc < HC; ++kc) {  // features 16 kc + 4 g .. + 3
        const floatx4 hv = ld4(hr + kc * 16);
        float v[4] = {hv[0], hv[1], hv[2], hv[3]};
#pragma unroll
        for (int lvl = 0; lvl < 3; ++lvl) {
            const unsigned int a = cvt_pk_bf16(v[0], v[1]), c = cvt_pk_bf16(v[2], v[3]);
            *reinterpret_cast<uint2*>(hq + lvl * 32 + 8 * kc) = make_uint2(a, c);
            if (lvl < 2) {
                v[0] -= __uint_as_float(a << 16);
                v[1] -= __uint_as_float(a & 0xFFFF0000u);
                v[2] -= __uint_as_float(c << 16);
                v[3] -= __uint_as_float(c & 0xFFFF0000u);
            }
        }
    }
}

// ---- env lanes (half-wave per env; v2 / v7) -----------------------------------------------------
struct EnvLane {
    UnitLane u;
    int e, b, st, slot, len, h0, act;
    int zcur;  // full-write tail: next row to zero (bits 0-15), exclusive end of the rows to zero (bits 16-30)
    uint32_t ep;
    float ret;
    bool stepped;
};

struct EnvCtx {
    const MlgEnvSpec* spec;
    const SpecShared* SS;
    UnitMasks M;
    RoEnv R;
    MlgBatch bt;
    MlgRunInfo info;
    const int* pairtab;
    const int* avtab;
    int* pk;   // [envs][32] packed unit states (pair pass)
    int* act;  // [envs][32] executed actions of the step (resolution)
    uint32_t* amask;  // [16] agents of env e that need a Q in the next agent phase (alive, env running)
    float* lobs;
    uint64_t* lavm;  // [16 envs * N] avail bit masks of the agents' current step
    int ldo, B;
    bool obf;  // v7: obs rows in LDS are bf16
    int U, N, A;  // env dims (compile-time constants in the static-shape v7 instantiations)
    bool sd;      // static dims: index tables replaced by arithmetic
    float inv_p;
};

__device__ __forceinline__ void env_observe(const EnvCtx& C, const MlgEnvSpec& spec, int slot, int t, int e, int hbase,
                                            int hl, const UnitLane& L, Stamps& sp) {
    v2_observe(C.M, spec, *C.SS, C.pairtab, C.avtab, C.bt, slot, t, e, hbase, hl, L, C.lobs, C.ldo, C.lavm, C.inv_p, sp,
               C.obf, C.U, C.N, C.A, C.sd);
}

__device__ inline void env_lane_reset(const EnvCtx& C, const MlgEnvState& st, EnvLane& E, int e, int e0, int hl) {
    const MlgEnvSpec& spec = *C.spec;
    const int hbase = (threadIdx.x & 63) & 32;
    E.e = e;
    E.b = e0 + e;
    E.u = UnitLane{0, 0, 0, 0u, 0u, 0};
    E.st = 2;
    E.slot = 0;
    E.len = 0;
    E.zcur = C.bt.T1;
    E.h0 = 0;
    E.act = 0;
    E.ep = 0;
    E.ret = 0.f;
    E.stepped = false;
    if (E.b < C.B) {  // reset (parallel_stepper.py:82-104; env_worker_process.py:54-60)
        E.ep = st.episode[E.b];
        E.st = 0;
        E.slot = C.bt.ring_size > 0 ? (C.bt.ring_slot0 + E.b) % C.bt.ring_size : E.b;
        E.zcur = tail_init(C.bt, E.slot);
        if (hl < C.U) {
            const int tm = C.SS->team[hl];
            env_spawn_xyh(make_tables(spec, *C.SS), mlg_env_key(spec.seed, E.b), E.ep, hl, C.SS->team_first[tm],
                          C.SS->team_size[tm], E.u.x, E.u.y, E.u.hp);
        }
        if (hl == 0) {
            st.episode[E.b] = E.ep + 1;
            gst(C.bt.filled + (int64_t)E.slot * C.bt.T1, (int64_t)1);
        }
    }
    if (hl == 0) {
        C.R.status[e] = E.st;
        C.R.slot[e] = E.slot;
        C.R.episode[e] = E.ep;
        C.amask[e] = E.b < C.B ? (C.N >= 32 ? 0xFFFFFFFFu : (1u << C.N) - 1u) : 0u;
    }
    if (E.b < C.B) {
        Stamps none;
        v2_pair_pass(C.M, C.U, hl, E.u, C.pk + e * 32);
        env_observe(C, spec, E.slot, 0, e, hbase, hl, E.u, none);
    }
}

// First half of env step t: record bookkeeping, executed actions (E1), resolution + moves (E2).
__device__ inline void env_lane_step1(const EnvCtx& C, EnvLane& E, int t, int hl) {
    E.stepped = false;
    if (E.st == 2) return;
    const MlgEnvSpec& spec = *C.spec;
    const int N = C.N, A = C.A, U = C.U, T1 = C.bt.T1;
    int* pact = C.R.pact + E.e * N;
    if (hl < N && !((C.amask[E.e] >> hl) & 1u)) {  // dead agent: no cell was run; its action is the no-op
        pact[hl] = 0;
        const int64_t off = ((int64_t)E.slot * T1 + t) * N + hl;
        gst(C.bt.actions + off, (int64_t)0);
        if (!C.bt.full_write) gst(C.bt.actions_onehot + off * A, 1.0f);
    }
    if (hl < N) C.R.prev[E.e * N + hl] = pact[hl];
    if (C.bt.full_write) {  // whole one-hot rows of the recorded actions
        const int64_t oh = ((int64_t)E.slot * T1 + t) * N * A;
        // rolled: the unrolled copy's rounded trip count was the v2 kernel's last VGPR spill, and its in-loop
        // scratch reload (vmcnt being in order) waited for every store of the step issued so far
#pragma unroll 1
        for (int k = hl; k < N * A; k += 32) {
            const int pt = C.sd ? ((k / A) << 8) | (k % A) : C.avtab[k];
            gst(C.bt.actions_onehot + oh + k, (pt & 255) == pact[pt >> 8] ? 1.0f : 0.0f);
        }
    }
    if (E.st == 1) {  // final action recorded; env done (parallel_stepper.py:153)
        E.st = 2;
        E.zcur = tail_start(E.zcur, t + 1);
        if (hl == 0) C.amask[E.e] = 0u;
        if (C.bt.full_write && hl == 0) {
            gst(C.bt.reward + (int64_t)E.slot * T1 + t, 0.f);
            gst(C.bt.terminated + (int64_t)E.slot * T1 + t, (uint8_t)0);
        }
        if (hl == 0) C.R.status[E.e] = E.st;
        return;
    }
    // E1: executed action -- validated policy action or the scripted AI choice (spec §3.4)
    const bool uvalid = hl < U;
    int act = 0;
    if (uvalid) {
        const int ag = C.SS->agent[hl];
        if (ag) {
            const int a = pact[ag - 1];
            act = (a >= 0 && a < MLG_ACT_BASE + U && v2_avail(C.M, spec.grid, E.u.x, E.u.y, E.u.hp, E.u.tgt, a)) ? a : 0;
        } else {
            act = E.u.ai;
        }
    }
    // E2: simultaneous resolution on the pre-step state, then moves (spec §3.4). Pre-step unit states are in
    // pk (written by the last pair pass), actions go through LDS too: 16-byte broadcast reads, no permutes.
    int* sact = C.act + E.e * 32;
    const int* spk = C.pk + E.e * 32;
    sact[hl] = act;
    int dmg = 0, heal = 0;
    resolve_hits(C.M, U, hl, spk, sact, dmg, heal);
    E.h0 = E.u.hp;
    if (uvalid && E.h0 > 0) {
        const int v = E.h0 - dmg + heal, mx = role_maxhp(mask_role(C.M, hl));
        E.u.hp = v < 0 ? 0 : (v > mx ? mx : v);
        E.u.x += (act == 3) - (act == 4);  // env_apply_move on registers
        E.u.y += (act == 1) - (act == 2);
    }
    E.act = act;
    E.stepped = true;
}

// Second half of env step t (envs that stepped): per-env reduction (E3), reward / termination, the
// observation of t + 1.
__device__ inline void env_lane_step2(const EnvCtx& C, EnvLane& E, int t, int hl, Stamps& sp) {
    if (!E.stepped) return;
    const MlgEnvSpec& spec = *C.spec;
    const int U = C.U, T1 = C.bt.T1;
    const int hbase = (threadIdx.x & 63) & 32;
    const bool uvalid = hl < U;
    const int h0 = E.h0, h1 = E.u.hp;
    const uint32_t alive_m = (uint32_t)(__ballot(uvalid && h1 > 0) >> hbase);
    const uint32_t kill_m = (uint32_t)(__ballot(uvalid && h0 > 0 && h1 == 0) >> hbase);
    int lost0, lost1;
    team_losses(C.M, uvalid && h0 > h1 ? h0 - h1 : 0, hbase, lost0, lost1);
    const int alive0 = __builtin_popcount(alive_m & ~C.M.team1), alive1 = __builtin_popcount(alive_m & C.M.team1);
    const int kills0 = __builtin_popcount(kill_m & C.M.team1), kills1 = __builtin_popcount(kill_m & ~C.M.team1);
    const int done = alive0 == 0 || alive1 == 0 || t + 1 >= spec.episode_limit;
    const int won0 = alive1 == 0 && alive0 > 0, won1 = alive0 == 0 && alive1 > 0;
    const int pt = spec.policy_team;
    const int wpt = pt ? won1 : won0, wop = pt ? won0 : won1;
    const int r_int = (pt ? lost0 : lost1) + 10 * (pt ? kills1 : kills0) + 200 * wpt;
    const float r = (float)r_int * 0.0625f;
    E.ret += r;
    if (hl == 0) {
        const int64_t sl = (int64_t)E.slot * T1 + t;
        gst(C.bt.reward + sl, r);
        gst(C.bt.terminated + sl, (uint8_t)done);
        gst(C.bt.filled + sl + 1, (int64_t)1);
        if (done) {
            gst(C.info.won + 2 * E.b, (int32_t)wpt);
            gst(C.info.won + 2 * E.b + 1, (int32_t)wop);
            gst(C.info.draw + E.b, (int32_t)(!won0 && !won1));
        }
    }
    if (done) {
        E.st = 1;
        E.len = t + 1;
    }
    if (hl == 0) C.R.status[E.e] = E.st;
    {  // agents alive after the step need a Q for the next action (incl. the final one after termination)
        const int N = C.N;
        const uint32_t am = (uint32_t)(__ballot(hl < N && ((alive_m >> C.SS->aunit[hl < N ? hl : 0]) & 1u)) >> hbase);
        if (hl == 0) C.amask[E.e] = am;
    }
    sp.mark(6);
    // observation at t + 1 (incl. envs that just terminated)
    v2_pair_pass(C.M, U, hl, E.u, C.pk + E.e * 32);
    sp.mark(7);
    env_observe(C, spec, E.slot, t + 1, E.e, hbase, hl, E.u, sp);
}

// Full-write mode: a finished env's half-wave zeroes a few more steps of its slot's tail.
__device__ inline void env_lane_tail(const EnvCtx& C, EnvLane& E, int steps, int hl) {
    const int z0 = E.zcur & 0xFFFF, zend = E.zcur >> 16;
    if (!C.bt.full_write || E.st != 2 || z0 >= zend || E.b >= C.B) return;
    const int z1 = z0 + steps < zend ? z0 + steps : zend;
    zero_slot_steps(C.bt, E.slot, z0, z1, C.N, C.A, 6 * C.U, 8 * C.U, hl, 32);
    E.zcur = (E.zcur & ~0xFFFF) | z1;
}

// Per-env summary + env state write-back (+ the rest of the tail in full-write mode).
__device__ inline void env_lane_finish(const EnvCtx& C, const MlgEnvState& st, EnvLane& E, int hl) {
    if (E.b >= C.B) return;
    const int U = C.U;
    if (C.bt.full_write) env_lane_tail(C, E, C.bt.T1, hl);
    if (hl == 0) {
        if (C.bt.full_write && C.bt.slot_extent) C.bt.slot_extent[E.slot] = E.len + 1;
        C.info.ep_len[E.b] = E.len;
        C.info.ret[E.b] = E.ret;
        st.t[E.b] = E.len;
    }
    if (hl < U) {
        st.x[(int64_t)E.b * U + hl] = E.u.x;
        st.y[(int64_t)E.b * U + hl] = E.u.y;
        st.hp[(int64_t)E.b * U + hl] = E.u.hp;
    }
}

__device__ inline EnvCtx make_env_ctx(const MlgEnvSpec& spec, const RolloutLds2& lay, int* smem, const MlgBatch& bt,
                                      const MlgRunInfo& info, int U, int N, int A, bool sd) {
    EnvCtx C;
    C.U = U;
    C.N = N;
    C.A = A;
    C.sd = sd;
    float* fm = reinterpret_cast<float*>(smem);
    C.spec = &spec;
    C.SS = reinterpret_cast<const SpecShared*>(smem + lay.env.spec);
    C.M = make_unit_masks(*C.SS, U);
    C.R = env_view(smem, lay.env);
    C.bt = bt;
    C.info = info;
    C.pairtab = smem + lay.pairtab;
    C.avtab = smem + lay.avtab;
    C.pk = smem + lay.pk;
    C.act = smem + lay.act;
    C.amask = reinterpret_cast<uint32_t*>(smem + lay.am);
    C.lobs = fm + lay.obs;
    C.lavm = reinterpret_cast<uint64_t*>(smem + lay.avail);
    C.ldo = lay.ldo;
    C.obf = lay.xpl != 0;
    C.B = bt.B;
    C.inv_p = 1.0f / (float)pow2_at_least(spec.grid);
    return C;
}

// Per-step copy of the env context for the env phase with the unit masks and the batch pointers moved into VGPRs
// behind an opaque asm: values derived from them (per-unit role / team predicates of the unrolled unit loops, store
// addresses) can then not be hoisted out of the step loop as loop invariants. Hoisted, they held ~40 SGPRs (64-bit
// lane masks per unit) across the loop and spilled, and every batch store reloaded the whole 16-SGPR pointer tuple
// from the spill lanes.
__device__ __forceinline__ EnvCtx env_ctx_step(const EnvCtx& C) {
    EnvCtx c = C;
    asm volatile("" : "+v"(c.M.team1), "+v"(c.M.healer), "+v"(c.M.tank), "+v"(c.M.melee));
    asm volatile("" : "+v"(c.bt.obs), "+v"(c.bt.state), "+v"(c.bt.avail), "+v"(c.bt.actions));
    asm volatile("" : "+v"(c.bt.actions_onehot), "+v"(c.bt.reward), "+v"(c.bt.terminated), "+v"(c.bt.filled));
    return c;
}

// ================================================================================================
// v2 kernel: 8 waves, 16 envs; every wave does agent work (chunk j = w % HC of tiles w / HC, ...) and then
// the env step of envs 2w, 2w + 1. Barriers per step: A|B, B|C, C|env, env|A.
// Static shape (SN agents, SU units > 0; v7 only): the agent and LDS layouts are compile-time constants (the
// headline 5v5 and the 3v3 plans, obs_last_action / obs_agent_id on), so their ~50 offsets are immediates instead
// of SGPRs -- the generic kernel spills SGPRs into VGPR lanes inside the step loop. Same code otherwise.
template <int H, bool G8, int SN, int SU>
struct StaticShape {
    static constexpr bool on = SN > 0;
    static constexpr MlgAgentDims dims{8 * SU, 5 + SU, SN, H, 8 * SU + 5 + SU + SN, 1, 1};
    static constexpr AgentLayout L = on ? make_agent_layout(dims) : AgentLayout{};
    static constexpr RolloutLds2 lay = on ? make_rollout_lds2(L, SU, SN, 16, 2, G8 ? 1 : 0) : RolloutLds2{};
};

// The batch pointers as eight independent SGPR pairs: loaded as one 16-SGPR tuple (s_load_dwordx16), a spilled
// tuple is reloaded whole (16 v_readlane) wherever any one pointer is used.
__device__ __forceinline__ MlgBatch split_batch_sgprs(MlgBatch b) {
    asm volatile("" : "+s"(b.obs), "+s"(b.state), "+s"(b.avail), "+s"(b.actions));
    asm volatile("" : "+s"(b.actions_onehot), "+s"(b.reward), "+s"(b.terminated), "+s"(b.filled));
    return b;
}

template <int H, bool G8, int SN = 0, int SU = 0>
__device__ __forceinline__ void rollout_v2_body(const MlgEnvSpec& spec, const MlgEnvState& st, const AgentLayout& L,
                                                const float* __restrict__ P, const MlgBatch& bt_arg, const MlgRunInfo& info,
                                                float eps, int test_mode, const RolloutLds2& lay, int DU, int DN,
                                                int DA, bool SD) {
    const MlgBatch bt = split_batch_sgprs(bt_arg);
    constexpr int HC = H / 16, NW = 8, REW = 16, G = NW / HC;
    extern __shared__ __attribute__((aligned(16))) int smem[];
    float* fm = reinterpret_cast<float*>(smem);
    const int N = spec.n_agents, lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hl = lane & 31;
    const int e0 = blockIdx.x * REW, T1 = bt.T1;
    v2_prologue(spec, L, P, lay, smem, REW * N);
    const EnvCtx C = make_env_ctx(spec, lay, smem, bt, info, DU, DN, DA, SD);
    EnvLane E;
    env_lane_reset(C, st, E, wave * 2 + (lane >> 5), e0, hl);
    const int j = wave % HC, gi = wave / HC;
    GruChunk<G8 ? 16 : H> W;  // v7 (G8) holds the split-bf16 weights of its 8 features instead
    GruG8 W8;
    if constexpr (G8)
        load_gru_g8(W8, P, L, lay, wave, lane);
    else
        load_gru_chunk<H>(W, P, L, fm, lay, j, lane);
    __syncthreads();
    Stamps sp;
    sp.init();
    uint64_t rows_issued = 0;  // agent rows issued to the MFMA cell (incl. tile padding)
    uint32_t m_prev = 0u;      // v7 row map of the previous step (make_rmap)
    int x_prev = 0;
    for (int t = 0; t < T1; ++t) {
        const uint32_t run = (uint32_t)__ballot(lane < REW && C.R.status[lane & (REW - 1)] < 2);
        sp.step(t, __popc(run));
        if (run == 0) break;
        // v7: one in-place buffer (nhb = 1); v2: double buffered by step parity
        const float* hc = fm + lay.hb + (t & 1) * (lay.nhb - 1) * lay.hsz;
        float* hn = fm + lay.hb + ((t & 1) ^ 1) * (lay.nhb - 1) * lay.hsz;
        StepRows SR;
        int tiles;
        int* wmap = smem + lay.rmap + wave * lay.rms;
        if constexpr (G8) {
            // rebuilt every step (skipping unchanged maps measured slower: the extra live registers spill)
            tiles = make_rmap(C.amask[lane & 15], wmap, lane, m_prev, x_prev);
            sp.mark(14);  // v7 stamps: row map (incl. the step's status ballot) in slot 14
            if constexpr (SN > 0) {
                const int nu = tiles > gi ? (tiles - gi + G - 1) / G : 0;
                fc1_g8_static<H, (8 * SU + 31) / 32, (SN + G - 1) / G>(L, lay, fm, wmap, C.R.prev, nu, j, gi, G, t, lane);
            } else
                ph_fc1_g8<H>(L, lay, fm, wmap, C.R.prev, tiles, j, gi, G, t, lane);
        } else {
            SR = make_rows(C.amask, 0, 16, lane);
            tiles = SR.tiles;
            ph_fc1<H>(L, lay, fm, C.R.prev, SR, j, gi, G, t, lane);
        }
        rows_issued += tiles * 16;
        sp.mark(0);
        lds_barrier();
        if constexpr (G8) sp.mark(5);  // v7 stamps: barrier A wait in slot 5, barrier B wait in slot 13
        int pre = -1;  // v7: epsilon coin of the wave's fc2 tile, drawn here (VALU next to the GRU's MFMAs)
        if constexpr (G8)
            if (wave < tiles) pre = eps_coin(spec, C.R, wmap, wave, e0, t, eps, test_mode, lane);
        if constexpr (G8)
            ph_gru_g8<H>(W8, lay, fm, wmap, hn, tiles, N, wave, lane);
        else
            ph_gru<H>(W, lay, fm, hc, hn, SR, N, j, gi, G, lane);
        sp.mark(1);
        lds_barrier();
        if constexpr (G8) sp.mark(13);
        if constexpr (G8)
            ph_fc2_g8<H>(spec, L, lay, fm, wmap, C.R, bt, hn, tiles, wave, NW, e0, t, eps, test_mode, lane, pre);
        else
            ph_fc2<H>(spec, L, lay, fm, C.R, bt, hn, SR, wave, NW, e0, t, eps, test_mode, lane);
        // v7: h' planes (hpl_split_tile) by the waves that have no fc2 tile, beside the fc2 phase (when every wave has
        // one -- tiles >= 8, generic shapes -- by the fc2 waves after their tiles)
        if constexpr (G8) {
            const bool idle = tiles < NW;
            const int step = idle ? NW - tiles : NW;
            for (int ti = idle ? wave - tiles : wave; ti >= 0 && ti < tiles; ti += step)
                hpl_split_tile<H>(lay, fm, wmap, hn, ti, N, lane);
        }
        sp.mark(2);
        lds_barrier();
        sp.mark(3);
        const EnvCtx Ce = env_ctx_step(C);
        env_lane_step1(Ce, E, t, hl);
        sp.mark(4);
        env_lane_step2(Ce, E, t, hl, sp);
#if defined(MLG_V7_TAIL_MIXED)
        if (!E.stepped && (t & 1)) env_lane_tail(Ce, E, 8, hl);
#else
        // a finished env's half-wave zeroes its slot's tail only while its partner half is idle too: in a wave whose
        // other env still steps, the zeroing would run after that env's step (one instruction stream) and lengthen
        // the step of the whole workgroup (barrier-bound); deferred rows are zeroed once the wave is idle or at the end
        if (__ballot(E.stepped) == 0 && (t & 1)) env_lane_tail(Ce, E, 8, hl);
#endif
        sp.mark(8);
        lds_barrier();
        sp.mark(10);
    }
    sp.flush();
    if (threadIdx.x == 0 && info.agent_rows) atomicAdd(info.agent_rows, (unsigned long long)rows_issued);
    env_lane_finish(C, st, E, hl);
}

template <int H, bool G8 = false, int SN = 0, int SU = 0>
__global__ void __launch_bounds__(512, 2) rollout_v2_kernel(MlgEnvSpec spec, MlgEnvState st, AgentLayout L,
                                                           const float* __restrict__ P, MlgBatch bt, MlgRunInfo info,
                                                           float eps, int test_mode, RolloutLds2 lay) {
    using S = StaticShape<H, G8, SN, SU>;
    if constexpr (S::on)
        rollout_v2_body<H, G8, SN, SU>(spec, st, S::L, P, bt, info, eps, test_mode, S::lay, SU, SN, 5 + SU, true);
    else
        rollout_v2_body<H, G8>(spec, st, L, P, bt, info, eps, test_mode, lay, spec.U, spec.n_agents, spec.n_actions,
                               G8);  // v7 layouts hold no index tables (arithmetic indices)
}

#include "rollout_sp.inc"
#include "rollout_sp8.inc"

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
                     const AgentLayout& L, const Sides& sd, const MlgRunInfo& info, int tm, const RolloutLds& lay) {
    const size_t bytes = (size_t)lay.total * 4;
    auto kern = rollout_kernel<H, TPW, WLDS>;
    if (bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)bytes);
        if (e != hipSuccess) return mlg::fail("rollout: LDS attribute (%zu B): %s", bytes, hipGetErrorString(e));
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), bytes, s, spec, st, L, sd, info, tm, lay);
    return 0;
}

// Weights in LDS when one policy's image fits (self-play holds two policies: weights stay in HBM / L2).
template <int H, int TPW>
int launch_rollout(int grid, int threads, hipStream_t s, const MlgEnvSpec& spec, const MlgEnvState& st,
                   const AgentLayout& L, const Sides& sd, const MlgRunInfo& info, int tm) {
    RolloutLds lay = make_rollout_lds(L, spec.U, spec.n_agents, true);
    if (sd.ns == 1 && lay.total * 4 <= LDS_LIMIT_BYTES && !getenv("MLG_ROLLOUT_GLOBAL_WEIGHTS"))
        return launch_rollout_t<H, TPW, true>(grid, threads, s, spec, st, L, sd, info, tm, lay);
    lay = make_rollout_lds(L, spec.U, spec.n_agents, false);
    return launch_rollout_t<H, TPW, false>(grid, threads, s, spec, st, L, sd, info, tm, lay);
}

// v7 with a compile-time shape when the layout matches one (StaticShape), else the generic v7.
template <int SN, int SU>
bool static_shape_matches(const AgentLayout& L, const RolloutLds2& lay) {
    using S = StaticShape<64, true, SN, SU>;
    return memcmp(&L, &S::L, sizeof(AgentLayout)) == 0 && memcmp(&lay, &S::lay, sizeof(RolloutLds2)) == 0;
}

template <int H, int V>
int launch_rollout_v2(hipStream_t s, const MlgEnvSpec& spec, const MlgEnvState& st, const AgentLayout& L,
                      const float* P, const MlgBatch& bt, const MlgRunInfo& info, float eps, int tm,
                      const RolloutLds2& lay) {
    const size_t bytes = (size_t)lay.total * 4;
    auto kern = V == 7 ? rollout_v2_kernel<64, true> : rollout_v2_kernel<H>;
    if (V == 7 && !getenv("MLG_ROLLOUT_GENERIC")) {
        if (static_shape_matches<5, 10>(L, lay)) kern = rollout_v2_kernel<64, true, 5, 10>;
        else if (static_shape_matches<3, 6>(L, lay)) kern = rollout_v2_kernel<64, true, 3, 6>;
    }
    const int threads = 512, rew = 16;
    if (bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)bytes);
        if (e != hipSuccess) return mlg::fail("rollout v2: LDS attribute (%zu B): %s", bytes, hipGetErrorString(e));
    }
    hipLaunchKernelGGL(kern, dim3((bt.B + rew - 1) / rew), dim3(threads), bytes, s, spec, st, L, P, bt, info, eps, tm,
                       lay);
    return 0;
}

// v7 for H = 64 and v2 for H = 32 when the shape allows it (U <= 32, LDS fits), else v1. MLG_ROLLOUT_KERNEL=
// v1|v2|v7 forces a variant (v1: the reference restatement, v2: fp32 compacted; both kept for the bit-identity tests).
int pick_rollout(const AgentLayout& L, const MlgEnvSpec& spec, RolloutLds2* lay) {
    const char* k = getenv("MLG_ROLLOUT_KERNEL");
    const int want = (k && k[0] == 'v') ? k[1] - '0' : (L.H == 64 ? 7 : 2);
    if (want == 1 || (L.H != 64 && L.H != 32) || spec.U > 32) return 1;
    *lay = make_rollout_lds2(L, spec.U, spec.n_agents, 16);
    if (lay->total * 4 > LDS_LIMIT_BYTES) return 1;
    if (want == 7 && L.H == 64) {
        *lay = make_rollout_lds2(L, spec.U, spec.n_agents, 16, 2, 1);
        if (lay->total * 4 <= LDS_LIMIT_BYTES) return 7;
        *lay = make_rollout_lds2(L, spec.U, spec.n_agents, 16);
    }
    return 2;
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

namespace {

int check_rollout_batch(const MlgBatch* batch, const MlgEnvSpec* spec, const MlgEnvState* st, const char* who) {
    MLG_REQUIRE(batch, "%s: null batch", who);
    MLG_REQUIRE(batch->state && batch->obs && batch->actions && batch->avail && batch->reward && batch->terminated &&
                    batch->actions_onehot && batch->filled,
                "%s: batch has null tensors", who);
    MLG_REQUIRE(batch->B == st->B, "%s: batch B=%d != env B=%d", who, batch->B, st->B);
    MLG_REQUIRE(batch->rows == nullptr, "%s: sampled (rows) views are read-only; use ring mode to write slots", who);
    MLG_REQUIRE(batch->T1 == spec->episode_limit + 1, "%s: batch T1=%d != episode_limit+1=%d", who, batch->T1,
                spec->episode_limit + 1);
    MLG_REQUIRE(batch->ring_size == 0 || (batch->ring_size >= batch->B && batch->ring_slot0 >= 0 &&
                                          batch->ring_slot0 < batch->ring_size),
                "%s: bad ring (slot0=%d size=%d B=%d)", who, batch->ring_slot0, batch->ring_size, batch->B);
    return 0;
}

// The generic (v1) kernel: any H in {32, 64, 128}, one or two policy sides.
int dispatch_rollout_v1(hipStream_t s, const MlgEnvSpec& spec, const MlgEnvState& st, const AgentLayout& L,
                        const Sides& sd, const MlgRunInfo& info, int test_mode) {
    const int tiles = sd.ns * ((RE * sd.nh + 15) / 16);
    const int W = tiles < 8 ? tiles : 8;
    const int tpw = (tiles + W - 1) / W;
    const int grid = (st.B + RE - 1) / RE;
    const int threads = W * 64;
    int rc = 0;
    MLG_REQUIRE(tpw <= 4, "rollout: %d agent tiles per wave > 4 (too many agents per env)", tpw);
#define MLG_RO(HH, TT) rc = launch_rollout<HH, TT>(grid, threads, s, spec, st, L, sd, info, test_mode)
    if (L.H == 64) {
        if (tpw == 1) MLG_RO(64, 1);
        else if (tpw == 2) MLG_RO(64, 2);
        else if (tpw == 3) MLG_RO(64, 3);
        else MLG_RO(64, 4);
    } else if (L.H == 32) {
        if (tpw == 1) MLG_RO(32, 1);
        else if (tpw == 2) MLG_RO(32, 2);
        else if (tpw == 3) MLG_RO(32, 3);
        else MLG_RO(32, 4);
    } else if (L.H == 128) {
        if (tpw == 1) MLG_RO(128, 1);
        else if (tpw == 2) MLG_RO(128, 2);
        else if (tpw == 3) MLG_RO(128, 3);
        else MLG_RO(128, 4);
    } else {
        return mlg::fail("rollout: rnn_hidden_dim=%d unsupported (32, 64, 128)", L.H);
    }
#undef MLG_RO
    if (rc) return rc;
    return mlg::check_launch("rollout_kernel");
}

}  // namespace

extern "C" int mlg_rollout(const MlgEnvSpec* spec, MlgEnvState* st, const MlgAgentDims* dims, const float* packed,
                           MlgBatch* batch, MlgRunInfo* info, float epsilon, int32_t test_mode, void* stream) {
    if (check_spec(spec) || check_state(st) || check_agent_dims(dims)) return 1;
    MLG_REQUIRE(packed && batch && info, "rollout: null pointer");
    if (check_rollout_batch(batch, spec, st, "rollout")) return 1;
    MLG_REQUIRE(info->ep_len && info->ret && info->won && info->draw, "rollout: run info has null tensors");
    MLG_REQUIRE(dims->n_agents == spec->n_agents && dims->n_actions == spec->n_actions && dims->d_obs == 8 * spec->U,
                "rollout: agent dims do not match env spec (N=%d/%d A=%d/%d d_obs=%d/%d)", dims->n_agents,
                spec->n_agents, dims->n_actions, spec->n_actions, dims->d_obs, 8 * spec->U);
    const AgentLayout L = make_agent_layout(*dims);
    hipStream_t s = (hipStream_t)stream;
    const float eps = test_mode ? 0.f : epsilon;
    RolloutLds2 lay2;
    const int variant = pick_rollout(L, *spec, &lay2);
    if (variant > 1) {
        const bool h64 = dims->hidden == 64;
        int rc = 0;
#define MLG_V(VV) rc = h64 ? launch_rollout_v2<64, VV>(s, *spec, *st, L, packed, *batch, *info, eps, test_mode, lay2) \
                           : launch_rollout_v2<32, VV>(s, *spec, *st, L, packed, *batch, *info, eps, test_mode, lay2)
        if (variant == 7) rc = launch_rollout_v2<64, 7>(s, *spec, *st, L, packed, *batch, *info, eps, test_mode, lay2);
        else MLG_V(2);
#undef MLG_V
        if (rc) return rc;
        return mlg::check_launch("rollout_v2_kernel");
    }
    Sides sd;
    sd.bt[0] = sd.bt[1] = *batch;
    sd.P[0] = sd.P[1] = packed;
    sd.eps[0] = sd.eps[1] = eps;
    sd.ns = 1;
    sd.nh = spec->n_agents;
    return dispatch_rollout_v1(s, *spec, *st, L, sd, *info, test_mode);
}

extern "C" int mlg_rollout_selfplay(const MlgEnvSpec* spec, MlgEnvState* st, const MlgAgentDims* dims,
                                    const float* home_packed, const float* away_packed, MlgBatch* home, MlgBatch* away,
                                    MlgRunInfo* info, float eps_home, float eps_away, int32_t test_mode, void* stream) {
    if (check_spec(spec) || check_state(st) || check_agent_dims(dims)) return 1;
    MLG_REQUIRE(home_packed && away_packed && info, "rollout_selfplay: null pointer");
    if (check_rollout_batch(home, spec, st, "rollout_selfplay (home)") ||
        check_rollout_batch(away, spec, st, "rollout_selfplay (away)"))
        return 1;
    MLG_REQUIRE(info->ep_len && info->ret && info->won && info->draw, "rollout_selfplay: run info has null tensors");
    MLG_REQUIRE(spec->n_policy_teams == 2 && spec->n_agents % 2 == 0,
                "rollout_selfplay: %d agents in %d policy teams do not fit the symmetric two-team scenario "
                "(stepper_utils.py:9)", spec->n_agents, spec->n_policy_teams);
    const int nh = spec->n_agents / 2;
    MLG_REQUIRE(dims->n_agents == nh && dims->n_actions == spec->n_actions && dims->d_obs == 8 * spec->U,
                "rollout_selfplay: agent dims do not match one side of the env (N=%d/%d A=%d/%d d_obs=%d/%d)",
                dims->n_agents, nh, dims->n_actions, spec->n_actions, dims->d_obs, 8 * spec->U);
    for (int a = 0; a < nh; ++a)
        MLG_REQUIRE(spec->team[spec->agent_unit[a]] == spec->policy_team &&
                        spec->team[spec->agent_unit[nh + a]] == 1 - spec->policy_team,
                    "rollout_selfplay: agents 0..%d must be the home team, %d..%d the away team", nh - 1, nh,
                    2 * nh - 1);
    const AgentLayout L = make_agent_layout(*dims);
    Sides sd;
    sd.bt[0] = *home;
    sd.bt[1] = *away;
    sd.P[0] = home_packed;
    sd.P[1] = away_packed;
    sd.eps[0] = test_mode ? 0.f : eps_home;
    sd.eps[1] = test_mode ? 0.f : eps_away;
    sd.ns = 2;
    sd.nh = nh;
    // self-play kernels (two policies): sp8 (one round of 16-env workgroups) for the static 5v5 / 3v3 self-play shapes
    // at H = 64, else sp7 (v7 agent phases, 8 envs per workgroup) for H = 64, else sp2 (v2 structure) when the shape
    // allows it, else the generic v1 kernel. MLG_ROLLOUT_KERNEL=v1 | sp2 | sp7 forces one.
    const char* k = getenv("MLG_ROLLOUT_KERNEL");
    const bool force_v1 = k && k[0] == 'v' && k[1] == '1', force_sp2 = k && !strcmp(k, "sp2");
    const bool force_sp7 = k && !strcmp(k, "sp7");
    if (!force_v1 && !force_sp2 && !force_sp7 && L.H == 64 && !getenv("MLG_ROLLOUT_GENERIC")) {
        void (*kern8)(MlgEnvSpec, MlgEnvState, const float*, const float*, MlgBatch, MlgBatch, MlgRunInfo, float, float,
                      int) = nullptr;
        size_t bytes = 0;
        if (static_shape_matches_sp8<10, 10>(L, spec->n_agents)) {
            kern8 = rollout_sp8_kernel<10, 10>;
            bytes = (size_t)StaticShapeSP8<10, 10>::lay.total * 4;
        } else if (static_shape_matches_sp8<6, 6>(L, spec->n_agents)) {
            kern8 = rollout_sp8_kernel<6, 6>;
            bytes = (size_t)StaticShapeSP8<6, 6>::lay.total * 4;
        }
        if (kern8) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern8),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
            if (e != hipSuccess)
                return mlg::fail("rollout_selfplay: LDS attribute (%zu B): %s", bytes, hipGetErrorString(e));
            hipLaunchKernelGGL(kern8, dim3((st->B + RS8 - 1) / RS8), dim3(512), bytes, (hipStream_t)stream, *spec, *st,
                               home_packed, away_packed, *home, *away, *info, sd.eps[0], sd.eps[1], test_mode);
            return mlg::check_launch("rollout_sp8_kernel");
        }
    }
    const RolloutLdsSP l7 = make_rollout_lds_sp(L, spec->U, spec->n_agents, true);
    if (!force_v1 && !force_sp2 && L.H == 64 && L.Dob <= 32 * SP7_MAXKK && l7.total * 4 <= LDS_LIMIT_BYTES) {
        const size_t bytes = (size_t)l7.total * 4;
        auto kern = rollout_sp7_kernel<0, 0>;  // runtime shapes; the 5v5 / 3v3 self-play plans as constants
        if (!getenv("MLG_ROLLOUT_GENERIC")) {
            if (static_shape_matches_sp<10, 10>(L, l7)) kern = rollout_sp7_kernel<10, 10>;
            else if (static_shape_matches_sp<6, 6>(L, l7)) kern = rollout_sp7_kernel<6, 6>;
        }
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        if (e != hipSuccess) return mlg::fail("rollout_selfplay: LDS attribute (%zu B): %s", bytes, hipGetErrorString(e));
        hipLaunchKernelGGL(kern, dim3((st->B + RS - 1) / RS), dim3(512), bytes, (hipStream_t)stream, *spec, *st, L,
                           home_packed, away_packed, *home, *away, *info, sd.eps[0], sd.eps[1], test_mode, l7);
        return mlg::check_launch("rollout_sp7_kernel");
    }
    const RolloutLdsSP lsp = make_rollout_lds_sp(L, spec->U, spec->n_agents);
    if (!force_v1 && (L.H == 64 || L.H == 32) && spec->U <= 32 && lsp.total * 4 <= LDS_LIMIT_BYTES) {
        const size_t bytes = (size_t)lsp.total * 4;
        auto kern = L.H == 64 ? rollout_sp_kernel<64> : rollout_sp_kernel<32>;
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        if (e != hipSuccess) return mlg::fail("rollout_selfplay: LDS attribute (%zu B): %s", bytes, hipGetErrorString(e));
        hipLaunchKernelGGL(kern, dim3((st->B + RS - 1) / RS), dim3(512), bytes, (hipStream_t)stream, *spec, *st, L,
                           home_packed, away_packed, *home, *away, *info, sd.eps[0], sd.eps[1], test_mode, lsp);
        return mlg::check_launch("rollout_sp_kernel");
    }
    return dispatch_rollout_v1((hipStream_t)stream, *spec, *st, L, sd, *info, test_mode);
}
