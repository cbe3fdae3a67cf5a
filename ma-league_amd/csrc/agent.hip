// agent.hip -- agent-side entry points: weight packing, DRQN forward over arbitrary rows,
// BasicMAC.forward from an EpisodeBatch, epsilon-greedy selection, QMixer forward.
#include "agent_device.h"
#include "mlg_host.h"

namespace {

// One thread per packed float: canonical nn.Module tensors -> kernel layout (agent_device.h).
__global__ void pack_agent_kernel(AgentLayout L, MlgAgentParams p, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.total) return;
    out[i] = pack_agent_elem(L, p, i);
}

// DRQN forward over R rows; one wave per 16-row tile.  DENSE: inputs[R][d_in].
// MAC mode: rows = (b, n) of an EpisodeBatch at time t, inputs built from obs / actions_onehot(t-1) / id.
template <int H, bool DENSE>
__global__ void __launch_bounds__(256) agent_forward_kernel(AgentLayout L, const float* __restrict__ P,
                                                           const float* __restrict__ inputs, MlgBatch bt, int t,
                                                           const float* __restrict__ h_in, float* __restrict__ q,
                                                           float* __restrict__ h_out, int R) {
    constexpr int HC = H / 16;
    const int lane = threadIdx.x & 63;
    const int tile = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (tile * 16 >= R) return;  // whole wave exits together
    const int col = lane & 15, g = lane >> 4;
    const int row = tile * 16 + col;
    const bool valid = row < R;
    RowIn in;
    in.prev_action = -1;
    if (DENSE) {
        in.x = valid ? inputs + (int64_t)row * L.d_in : nullptr;
        in.onehot = nullptr;
        in.agent = 0;
    } else {
        const int N = L.N, b = row / N, n = row % N;
        const int64_t off = ((bt.rows ? (int64_t)bt.rows[b] : (int64_t)b) * bt.T1 + t) * N + n;
        in.x = valid ? bt.obs + off * L.d_obs : nullptr;
        in.onehot = (valid && t > 0) ? bt.actions_onehot + (off - N) * L.A : nullptr;
        in.agent = valid ? n : 0;
    }
    floatx4 h[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) {
        floatx4 v = {0.f, 0.f, 0.f, 0.f};
        if (valid && h_in) v = ld4(h_in + (int64_t)row * H + c * 16 + 4 * g);
        h[c] = v;
    }
    const WView W = global_view(P, L);
    agent_cell_hidden<H, DENSE>(W, L, in, h, lane);
    if (valid) {
#pragma unroll
        for (int c = 0; c < HC; ++c) *reinterpret_cast<floatx4*>(h_out + (int64_t)row * H + c * 16 + 4 * g) = h[c];
    }
    for (int at = 0; at < L.Ap / 16; ++at) {
        const floatx4 qt = agent_q_tile<H>(W, h, at, lane);
        if (!valid) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int a = at * 16 + 4 * g + r;
            if (a < L.A) q[(int64_t)row * L.A + a] = qt[r];
        }
    }
}

__global__ void select_actions_kernel(const float* __restrict__ q, const int32_t* __restrict__ avail, int R, int A,
                                      int n_agents, const uint64_t* __restrict__ keys, const uint32_t* __restrict__ episodes,
                                      int t, float eps, int64_t* __restrict__ actions, int64_t* __restrict__ is_greedy) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const float* qr = q + (int64_t)r * A;
    const int32_t* ar = avail + (int64_t)r * A;
    float bv = -INFINITY;
    int bi = 1 << 30;
    for (int a = 0; a < A; ++a) {
        const float v = ar[a] == 0 ? -INFINITY : qr[a];
        if (amax_better(v, a, bv, bi)) { bv = v; bi = a; }
    }
    int act = bi;
    int greedy = 1;
    if (eps > 0.f && keys) {
        const int env = r / n_agents, n = r % n_agents;
        const uint32_t ep = episodes ? episodes[env] : 0u;
        const uint64_t r1 = mlg_rng(keys[env], mlg_ctr(ep, (uint32_t)t, MLG_PURPOSE_EPS, (uint32_t)n));
        if (mlg_u01(r1) < eps) {
            greedy = 0;
            act = random_available(ar, A, mlg_rng(keys[env], mlg_ctr(ep, (uint32_t)t, MLG_PURPOSE_RAND, (uint32_t)n)));
        }
    }
    actions[r] = act;
    if (is_greedy) is_greedy[r] = greedy;
}

// ---- QMixer forward (qmix.py:41-59), one thread per row; used by QMixer.forward outside training ----
struct QMixP {
    MlgQMixParams p;
};

__device__ float lin_row(const float* w, const float* b, const float* x, int K, int o) {
    float acc = b[o];
    for (int k = 0; k < K; ++k) acc = fmaf(w[(int64_t)o * K + k], x[k], acc);
    return acc;
}

__global__ void qmix_forward_kernel(MlgQMixParams p, const float* __restrict__ qs, const float* __restrict__ states,
                                    float* __restrict__ out, int R) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const int N = p.n_agents, S = p.state_dim, E = p.embed_dim, HE = p.hypernet_embed;
    const float* s = states + (int64_t)r * S;
    const float* q = qs + (int64_t)r * N;
    float hid[64];
    float hb[256];
    // hidden = elu(q . |W1(s)| + b1(s))
    if (p.hypernet_layers == 2)
        for (int k = 0; k < HE; ++k) hb[k] = fmaxf(lin_row(p.hw1_0w, p.hw1_0b, s, S, k), 0.f);
    for (int e = 0; e < E; ++e) {
        float acc = 0.f;
        for (int n = 0; n < N; ++n) {
            const int o = n * E + e;
            const float w = p.hypernet_layers == 2 ? lin_row(p.hw1_2w, p.hw1_2b, hb, HE, o) : lin_row(p.hw1_0w, p.hw1_0b, s, S, o);
            acc = fmaf(q[n], fabsf(w), acc);
        }
        const float pre = acc + lin_row(p.hb1_w, p.hb1_b, s, S, e);
        hid[e] = pre > 0.f ? pre : expm1f(pre);
    }
    if (p.hypernet_layers == 2)
        for (int k = 0; k < HE; ++k) hb[k] = fmaxf(lin_row(p.hwf_0w, p.hwf_0b, s, S, k), 0.f);
    float y = 0.f;
    for (int e = 0; e < E; ++e) {
        const float w = p.hypernet_layers == 2 ? lin_row(p.hwf_2w, p.hwf_2b, hb, HE, e) : lin_row(p.hwf_0w, p.hwf_0b, s, S, e);
        y = fmaf(hid[e], fabsf(w), y);
    }
    float hv[64];
    for (int e = 0; e < E; ++e) hv[e] = fmaxf(lin_row(p.v0_w, p.v0_b, s, S, e), 0.f);
    const float v = lin_row(p.v2_w, p.v2_b, hv, E, 0);
    out[r] = y + v;
}

}  // namespace

int check_agent_dims(const MlgAgentDims* d) {
    MLG_REQUIRE(d != nullptr, "null agent dims");
    MLG_REQUIRE(d->hidden == 32 || d->hidden == 64 || d->hidden == 128, "rnn_hidden_dim=%d unsupported (32/64/128)",
                d->hidden);
    MLG_REQUIRE(d->n_actions >= 1 && d->n_agents >= 1 && d->d_obs >= 1, "invalid agent dims");
    const int expect = d->d_obs + (d->obs_last_action ? d->n_actions : 0) + (d->obs_agent_id ? d->n_agents : 0);
    MLG_REQUIRE(d->d_in == expect, "agent d_in=%d does not match obs/last-action/id layout (%d)", d->d_in, expect);
    return 0;
}

extern "C" int64_t mlg_packed_agent_size(const MlgAgentDims* d) {
    if (check_agent_dims(d)) return -1;
    return make_agent_layout(*d).total;
}

extern "C" int mlg_pack_agent(const MlgAgentDims* d, const MlgAgentParams* p, float* packed, void* stream) {
    if (check_agent_dims(d)) return 1;
    MLG_REQUIRE(p && p->fc1_w && p->fc1_b && p->w_ih && p->b_ih && p->w_hh && p->b_hh && p->fc2_w && p->fc2_b && packed,
                "pack_agent: null pointer");
    const AgentLayout L = make_agent_layout(*d);
    hipLaunchKernelGGL(pack_agent_kernel, dim3((unsigned)((L.total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, L, *p,
                       packed);
    return mlg::check_launch("pack_agent_kernel");
}

namespace {
template <bool DENSE>
int launch_forward(const MlgAgentDims* d, const float* packed, const float* inputs, const MlgBatch& bt, int t,
                   const float* h_in, float* q, float* h_out, int R, hipStream_t s) {
    const AgentLayout L = make_agent_layout(*d);
    const int tiles = (R + 15) / 16;
    const int grid = (tiles + 3) / 4;
    if (R == 0) return 0;
    if (d->hidden == 64)
        hipLaunchKernelGGL((agent_forward_kernel<64, DENSE>), dim3(grid), dim3(256), 0, s, L, packed, inputs, bt, t, h_in, q,
                           h_out, R);
    else if (d->hidden == 32)
        hipLaunchKernelGGL((agent_forward_kernel<32, DENSE>), dim3(grid), dim3(256), 0, s, L, packed, inputs, bt, t, h_in, q,
                           h_out, R);
    else
        hipLaunchKernelGGL((agent_forward_kernel<128, DENSE>), dim3(grid), dim3(256), 0, s, L, packed, inputs, bt, t, h_in,
                           q, h_out, R);
    return mlg::check_launch("agent_forward_kernel");
}
}  // namespace

extern "C" int mlg_agent_forward(const MlgAgentDims* d, const float* packed, const float* inputs, const float* h_in,
                                 float* q, float* h_out, int32_t R, void* stream) {
    if (check_agent_dims(d)) return 1;
    MLG_REQUIRE(packed && inputs && q && h_out && R >= 0, "agent_forward: bad arguments");
    MlgBatch none{};
    return launch_forward<true>(d, packed, inputs, none, 0, h_in, q, h_out, R, (hipStream_t)stream);
}

extern "C" int mlg_mac_forward(const MlgAgentDims* d, const float* packed, const MlgBatch* batch, int32_t t,
                               const float* h_in, float* q, float* h_out, void* stream) {
    if (check_agent_dims(d)) return 1;
    MLG_REQUIRE(packed && batch && batch->obs && batch->actions_onehot && q && h_out, "mac_forward: bad arguments");
    MLG_REQUIRE(t >= 0 && t < batch->T1, "mac_forward: t=%d out of [0, %d)", t, batch->T1);
    return launch_forward<false>(d, packed, nullptr, *batch, t, h_in, q, h_out, batch->B * d->n_agents,
                                 (hipStream_t)stream);
}

extern "C" int mlg_select_actions(const float* q, const int32_t* avail, int32_t R, int32_t A, int32_t n_agents,
                                  const uint64_t* keys, const uint32_t* episodes, int32_t t, float epsilon,
                                  int64_t* actions, int64_t* is_greedy, void* stream) {
    MLG_REQUIRE(q && avail && actions && R >= 0 && A >= 1 && n_agents >= 1, "select_actions: bad arguments");
    MLG_REQUIRE(epsilon <= 0.f || keys, "select_actions: epsilon > 0 needs rng keys");
    if (R == 0) return 0;
    hipLaunchKernelGGL(select_actions_kernel, dim3((R + 255) / 256), dim3(256), 0, (hipStream_t)stream, q, avail, R, A,
                       n_agents, keys, episodes, t, epsilon, actions, is_greedy);
    return mlg::check_launch("select_actions_kernel");
}

extern "C" int mlg_qmix_forward(const MlgQMixParams* p, const float* agent_qs, const float* states, float* q_tot,
                                int32_t R, void* stream) {
    MLG_REQUIRE(p && agent_qs && states && q_tot, "qmix_forward: null pointer");
    MLG_REQUIRE(p->embed_dim <= 64 && p->hypernet_embed <= 256, "qmix_forward: embed dims too large");
    MLG_REQUIRE(p->hypernet_layers == 1 || p->hypernet_layers == 2, "qmix_forward: hypernet_layers must be 1 or 2");
    if (R == 0) return 0;
    hipLaunchKernelGGL(qmix_forward_kernel, dim3((R + 127) / 128), dim3(128), 0, (hipStream_t)stream, *p, agent_qs, states,
                       q_tot, R);
    return mlg::check_launch("qmix_forward_kernel");
}

extern "C" const char* mlg_last_error(void) { return mlg::last_error().c_str(); }
extern "C" const char* mlg_version(void) { return "maleague-gfx950 0.1.0"; }
