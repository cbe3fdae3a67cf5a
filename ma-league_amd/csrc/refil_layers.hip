// refil_layers.hip -- layer-level REFIL entry points (the module forward()s of the Python classes and the
// kernels the reference's layer golden vectors are checked against):
//
//   mlg_refil_attention      EntityAttentionLayer.forward (+ backward) over bs items
//                            (src/marl/modules/layers/attention.py:24-79)
//   mlg_refil_pack_mixer     FlexQMixer named_parameters -> 4 packed AttentionHyperNet blocks
//   mlg_refil_mixer_forward  FlexQMixer.forward, plain or with imagine groups (src/marl/modules/mixers/
//                            flex_qmix.py:73-117)
// Same device building blocks as the rollout / learner (refil_device.h).
#include "mlg_host.h"
#include "refil_device.h"

using namespace refil;

namespace {

// ---- EntityAttentionLayer: one wave per item -------------------------------------------------------------
__global__ void __launch_bounds__(64) attention_kernel(const float* __restrict__ w_in, const float* __restrict__ w_out,
                                                       const float* __restrict__ b_out, const float* __restrict__ x,
                                                       const uint8_t* __restrict__ pre, const uint8_t* __restrict__ post,
                                                       int ne, int nq, float* __restrict__ y,
                                                       const float* __restrict__ gy, float* __restrict__ dx,
                                                       float* __restrict__ dw_in, float* __restrict__ dw_out,
                                                       float* __restrict__ db_out) {
    __shared__ float s_x[NE * LDX];
    __shared__ float s_qkv[NE * LDQ];
    __shared__ float s_o[16 * LDX];
    __shared__ float s_do[16 * LDX];
    __shared__ float s_dqkv[NE * LDQ];
    __shared__ float s_P[NH * 16 * NE];
    __shared__ float s_ds[NH * 16 * NE];
    __shared__ uint32_t s_m[16];
    __shared__ uint32_t s_dead;
    const int lane = threadIdx.x, it = blockIdx.x;
    const int col = lane & 15, g = lane >> 4;
    for (int i = lane; i < NE * EMB; i += 64) {
        const int j = i / EMB, c = i % EMB;
        s_x[j * LDX + c] = j < ne ? x[((int64_t)it * ne + j) * EMB + c] : 0.f;
    }
    for (int i = lane; i < 16 * LDX; i += 64) s_o[i] = 0.f;
    if (lane < 16) {
        uint32_t m = 0xFFFFFFFFu;
        if (lane < nq) {
            m = ~((1u << ne) - 1u);
            for (int j = 0; j < ne; ++j) m |= (uint32_t)(pre[((int64_t)it * nq + lane) * ne + j] != 0) << j;
        }
        s_m[lane] = m;
    }
    if (lane == 0) {
        uint32_t d = ~((1u << nq) - 1u) & 0xFFFFu;
        for (int q = 0; q < nq; ++q) d |= (uint32_t)(post[(int64_t)it * nq + q] != 0) << q;
        s_dead = d;
    }
    wave_sync();
    dense_lds<false>(w_in, EMB, nullptr, 3 * EMB / 16, s_x, LDX, EMB / 16, s_qkv, LDQ, lane);
    wave_sync();
    attn_fwd(s_qkv, s_m, nq, ne, s_o, LDX, s_P, lane);
    wave_sync();
    const bool rdead = (s_dead >> col) & 1u;
    floatx4 yv[4];
    bias_init<4>(yv, b_out, 0, lane);
    mm_lds<4>(yv, w_out, EMB, 0, s_o, LDX, EMB / 16, lane);
    if (col < nq) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<floatx4*>(y + ((int64_t)it * nq + col) * EMB + q * 16 + 4 * g) =
                rdead ? floatx4{0.f, 0.f, 0.f, 0.f} : yv[q];
    }
    if (!gy) return;
    // ---- backward: dout = gy * alive; dO = W_out^T dout; attention bwd; dx = W_in^T dqkv ----
    for (int i = lane; i < 16 * LDX; i += 64) s_do[i] = 0.f;
    wave_sync();
    for (int i = lane; i < nq * EMB; i += 64) {
        const int q = i / EMB, c = i % EMB;
        const float d = ((s_dead >> q) & 1u) ? 0.f : gy[((int64_t)it * nq + q) * EMB + c];
        atomicAdd(db_out + c, d);
        s_dqkv[q * LDQ + c] = d;  // scratch: dout rows
    }
    wave_sync();
    for (int i = lane; i < EMB * EMB; i += 64) {  // dW_out[m][k] += sum_q dout[q][m] o[q][k]
        const int m = i / EMB, k = i % EMB;
        float s = 0.f;
        for (int q = 0; q < nq; ++q) s += s_dqkv[q * LDQ + m] * s_o[q * LDX + k];
        atomicAdd(dw_out + i, s);
    }
    for (int i = lane; i < nq * EMB; i += 64) {  // dO[q][k] = sum_m dout[q][m] W_out[m][k]
        const int q = i / EMB, k = i % EMB;
        float s = 0.f;
        for (int m = 0; m < EMB; ++m) s += s_dqkv[q * LDQ + m] * w_out[m * EMB + k];
        s_do[q * LDX + k] = s;
    }
    wave_sync();
    attn_bwd<false>(s_qkv, s_P, nq, s_do, LDX, s_ds, s_dqkv, lane);
    wave_sync();
    for (int i = lane; i < 3 * EMB * EMB; i += 64) {  // dW_in[f][c] += sum_j dqkv[j][f] x[j][c]
        const int f = i / EMB, c = i % EMB;
        float s = 0.f;
        for (int j = 0; j < ne; ++j) s += s_dqkv[j * LDQ + f] * s_x[j * LDX + c];
        atomicAdd(dw_in + i, s);
    }
    for (int i = lane; i < ne * EMB; i += 64) {  // dx[j][c] = sum_f dqkv[j][f] W_in[f][c]
        const int j = i / EMB, c = i % EMB;
        float s = 0.f;
        for (int f = 0; f < 3 * EMB; ++f) s += s_dqkv[j * LDQ + f] * w_in[f * EMB + c];
        dx[((int64_t)it * ne + j) * EMB + c] = s;
    }
}

// ---- FlexQMixer forward: one workgroup (4 waves, wave k = hypernet k) per row ----------------------------------
struct CopyJob {
    int64_t src, dst;
    int rows_dst, cols_dst, rows_src, cols_src;
};

__global__ void pack_hyper_kernel(RHyper L, const float* __restrict__ flat, float* __restrict__ packed) {
    const int k = blockIdx.y;
    const float* src = flat + (int64_t)k * L.c_total;
    float* dst = packed + (int64_t)k * L.total;
    const CopyJob J[7] = {{L.c_w1, L.w1, EMB, L.K1, EMB, L.D0},         {L.c_b1, L.b1, 1, EMB, 1, EMB},
                          {L.c_win, L.win, 3 * EMB, EMB, 3 * EMB, EMB}, {L.c_wout, L.wout, EMB, EMB, EMB, EMB},
                          {L.c_bout, L.bout, 1, EMB, 1, EMB},           {L.c_w2, L.w2, EM, EMB, EM, EMB},
                          {L.c_b2, L.b2, 1, EM, 1, EM}};
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.total) return;
    float v = 0.f;
    for (int q = 0; q < 7; ++q) {
        const int64_t n = (int64_t)J[q].rows_dst * J[q].cols_dst;
        if (i >= J[q].dst && i < J[q].dst + n) {
            const int64_t l = i - J[q].dst;
            const int r = (int)(l / J[q].cols_dst), c = (int)(l % J[q].cols_dst);
            if (r < J[q].rows_src && c < J[q].cols_src) v = src[J[q].src + (int64_t)r * J[q].cols_src + c];
            break;
        }
    }
    dst[i] = v;
}

struct MixFwdArgs {
    int NA, NE, D0, R, softmax;
    const float* packed;  // 4 RHyper blocks
    const float* qs;      // [R][NA or 2 NA]
    const float* ent;     // [R][NE][D0]
    const uint8_t* em;    // [R][NE]
    const uint8_t* wm;    // [R][NE][NE] or null
    const uint8_t* im;
    float* out;           // [R]
};

__global__ void __launch_bounds__(256) mixer_fwd_kernel(RHyper L, MixFwdArgs a) {
    __shared__ float s_ein[NE * LDI];
    __shared__ float s_x1[4][NE * LDX];
    __shared__ float s_qkv[4][NE * LDQ];
    __shared__ float s_o[4][16 * LDX];
    __shared__ float s_X[5][NAS * EM];  // w1 (plain or W), w1 I, w_final, b1, V
    __shared__ uint32_t s_m[3][16];
    __shared__ uint32_t s_dead;
    const int tid = threadIdx.x, lane = tid & 63, k = tid >> 6;
    const int r = blockIdx.x;
    const bool imagine = a.wm != nullptr;
    for (int i = tid; i < NE * L.K1; i += blockDim.x) {
        const int j = i / L.K1, c = i % L.K1;
        s_ein[j * LDI + c] = (j < a.NE && c < a.D0) ? a.ent[((int64_t)r * a.NE + j) * a.D0 + c] : 0.f;
    }
    for (int i = tid; i < 4 * 16 * LDX; i += blockDim.x) (&s_o[0][0])[i] = 0.f;
    if (tid < 16) {
        const int q = tid;
        uint32_t em = ~((1u << a.NE) - 1u) & 0xFFFFu;
        for (int j = 0; j < a.NE; ++j) em |= (uint32_t)(a.em[(int64_t)r * a.NE + j] != 0) << j;
        const uint32_t dead = ((em & ((1u << a.NA) - 1u)) | ~((1u << a.NA) - 1u)) & 0xFFu;
        s_m[0][q] = (q < NAS && ((dead >> q) & 1u)) ? 0xFFFFu : em;
        if (imagine) {
            uint32_t w = ~((1u << a.NE) - 1u) & 0xFFFFu, im = w;
            if (q < a.NE) {
                for (int j = 0; j < a.NE; ++j) {
                    w |= (uint32_t)(a.wm[((int64_t)r * a.NE + q) * a.NE + j] != 0) << j;
                    im |= (uint32_t)(a.im[((int64_t)r * a.NE + q) * a.NE + j] != 0) << j;
                }
            } else {
                w = im = 0xFFFFu;
            }
            s_m[1][q] = w;
            s_m[2][q] = im;
        }
        if (q == 0) s_dead = dead;
    }
    __syncthreads();
    const float* P = a.packed + (int64_t)k * L.total;
    dense_lds<true>(P + L.w1, L.K1, P + L.b1, EMB / 16, s_ein, LDI, L.K1 / 16, s_x1[k], LDX, lane);
    wave_sync();
    dense_lds<false>(P + L.win, EMB, nullptr, 3 * EMB / 16, s_x1[k], LDX, EMB / 16, s_qkv[k], LDQ, lane);
    wave_sync();
    // hyper_w_1 with imagine groups: W and I masks; every other hypernet: the default entity mask
    const int V = (k == 0 && imagine) ? 2 : 1;
    for (int v = 0; v < V; ++v)
        attn_fwd(s_qkv[k], s_m[(k == 0 && imagine) ? v + 1 : 0], a.NA, a.NE, s_o[k] + v * NAS * LDX, LDX, nullptr,
                 lane);
    wave_sync();
    const int col = lane & 15, g = lane >> 4;
    const int v = col >> 3, n = col & 7;
    const bool rdead = (s_dead >> n) & 1u;
    floatx4 x2[4];
    bias_init<4>(x2, P + L.bout, 0, lane);
    mm_lds<4>(x2, P + L.wout, EMB, 0, s_o[k], LDX, EMB / 16, lane);
    if (rdead) {
#pragma unroll
        for (int q = 0; q < 4; ++q) x2[q] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    floatx4 X[2];
    bias_init<2>(X, P + L.b2, 0, lane);
    mm_reg<2, 4>(X, P + L.w2, EMB, 0, x2, lane);
    if (rdead) X[0] = X[1] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (v < V) {
        const int slot = k == 0 ? v : k + 1;
#pragma unroll
        for (int q = 0; q < 2; ++q) *reinterpret_cast<floatx4*>(&s_X[slot][n * EM + q * 16 + 4 * g]) = X[q];
    }
    __syncthreads();
    if (tid >= 32) return;
    // ---- mixing (flex_qmix.py:91-117), lane = embed index e ----
    const int e = tid;
    const int NA = a.NA, nrow = imagine ? 2 * NA : NA;
    auto sum32 = [](float x) {
#pragma unroll
        for (int m = 1; m < 32; m <<= 1) x += __shfl_xor(x, m, 32);
        return x;
    };
    auto mw = [&](float x) {
        if (!a.softmax) return fabsf(x);
        float m = x;
#pragma unroll
        for (int s = 1; s < 32; s <<= 1) m = fmaxf(m, __shfl_xor(m, s, 32));
        const float ex = expf(x - m);
        return ex / sum32(ex);
    };
    float b1 = 0.f, wfp = 0.f, vs = 0.f;
    for (int q = 0; q < NA; ++q) {
        b1 += s_X[3][q * EM + e];
        wfp += s_X[2][q * EM + e];
        vs += s_X[4][q * EM + e];
    }
    b1 /= (float)NA;
    const float wf = mw(wfp / (float)NA);
    float pre = b1;
    for (int q = 0; q < nrow; ++q) {
        const float xw = q < NA ? s_X[0][q * EM + e] : s_X[1][(q - NA) * EM + e];
        pre += a.qs[(int64_t)r * nrow + q] * mw(xw);
    }
    const float hid = pre > 0.f ? pre : expm1f(pre);
    const float y = sum32(hid * wf) + sum32(vs) / ((float)NA * (float)EM);
    if (e == 0) a.out[r] = y;
}

}  // namespace

extern "C" int mlg_refil_attention(const float* w_in, const float* w_out, const float* b_out, const float* x,
                                   const uint8_t* pre_mask, const uint8_t* post_mask, int32_t bs, int32_t ne, int32_t nq,
                                   int32_t n_heads, float* y, const float* gy, float* dx, float* dw_in, float* dw_out,
                                   float* db_out, void* stream) {
    MLG_REQUIRE(w_in && w_out && b_out && x && pre_mask && post_mask && y, "refil_attention: null pointer");
    MLG_REQUIRE(n_heads == NH, "refil_attention: attn_n_heads=%d unsupported (4; embed 64)", n_heads);
    MLG_REQUIRE(ne >= 1 && ne <= NE && nq >= 1 && nq <= 16 && nq <= ne, "refil_attention: ne=%d nq=%d (<= 16)", ne, nq);
    MLG_REQUIRE(!gy || (dx && dw_in && dw_out && db_out), "refil_attention: backward needs dx, dw_in, dw_out, db_out");
    if (bs <= 0) return 0;
    hipLaunchKernelGGL(attention_kernel, dim3((unsigned)bs), dim3(64), 0, (hipStream_t)stream, w_in, w_out, b_out, x,
                       pre_mask, post_mask, ne, nq, y, gy, dx, dw_in, dw_out, db_out);
    return mlg::check_launch("refil_attention");
}

static int check_mixer_dims(const MlgRefilDims* d) {
    MLG_REQUIRE(d != nullptr, "null refil dims");
    MLG_REQUIRE(d->n_agents >= 1 && d->n_agents <= NAS && d->n_entities >= d->n_agents && d->n_entities <= NE,
                "refil mixer: n_agents=%d n_entities=%d unsupported", d->n_agents, d->n_entities);
    const int D0 = d->entity_shape + (d->entity_last_action ? d->n_actions : 0);
    MLG_REQUIRE(D0 <= KMAX && d->attn_n_heads == NH, "refil mixer: entity input %d (<= %d), heads %d (4)", D0, KMAX,
                d->attn_n_heads);
    return 0;
}

extern "C" int64_t mlg_refil_packed_mixer_size(const MlgRefilDims* d) {
    if (check_mixer_dims(d)) return -1;
    return 4 * make_rhyper(d->entity_shape + (d->entity_last_action ? d->n_actions : 0)).total;
}

extern "C" int mlg_refil_pack_mixer(const MlgRefilDims* d, const float* flat, float* packed, void* stream) {
    if (check_mixer_dims(d)) return 1;
    MLG_REQUIRE(flat && packed, "refil_pack_mixer: null pointer");
    const RHyper L = make_rhyper(d->entity_shape + (d->entity_last_action ? d->n_actions : 0));
    hipLaunchKernelGGL(pack_hyper_kernel, dim3((unsigned)((L.total + 255) / 256), 4), dim3(256), 0, (hipStream_t)stream, L,
                       flat, packed);
    return mlg::check_launch("refil_pack_mixer");
}

extern "C" int mlg_refil_mixer_forward(const MlgRefilDims* d, const float* packed, const float* agent_qs,
                                       const float* entities, const uint8_t* entity_mask, const uint8_t* w_mask,
                                       const uint8_t* i_mask, int32_t softmax_mixing_weights, float* q_tot, int32_t R,
                                       void* stream) {
    if (check_mixer_dims(d)) return 1;
    MLG_REQUIRE(packed && agent_qs && entities && entity_mask && q_tot, "refil_mixer_forward: null pointer");
    MLG_REQUIRE((w_mask == nullptr) == (i_mask == nullptr), "refil_mixer_forward: imagine needs both W and I masks");
    if (R <= 0) return 0;
    const int D0 = d->entity_shape + (d->entity_last_action ? d->n_actions : 0);
    const RHyper L = make_rhyper(D0);
    MixFwdArgs a{d->n_agents, d->n_entities, D0, R, softmax_mixing_weights, packed, agent_qs, entities, entity_mask,
                 w_mask, i_mask, q_tot};
    hipLaunchKernelGGL(mixer_fwd_kernel, dim3((unsigned)R), dim3(256), 0, (hipStream_t)stream, L, a);
    return mlg::check_launch("refil_mixer_forward");
}
