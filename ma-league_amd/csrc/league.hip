// league.hip -- league bookkeeping on the device.
//
// mlg_league_record_runs: the episode results of one batched self-play run folded into the league's local payoff
// delta entry (home, away) in ONE launch, replacing a dozen elementwise / reduce launches of the host-side form.
// Restates _extract_result + _update_payoff (src/league/processes/training/league_experiment_process.py:85-105):
// per env, DRAW if the env says so or if both / no team won, else WIN / LOSS by the policy team's battle_won;
// GAMES += B unless the reference-compatible payoff is kept (the reference never increments GAMES, payoff.py).
#include <hip/hip_runtime.h>

#include "../../include/maleague.h"
#include "mlg_host.h"

namespace {

constexpr int kRecThreads = 1024;

// one block: lane-strided pass over the envs, wave ballots, a 16-wave LDS sum, thread 0 adds into the entry
__global__ void __launch_bounds__(kRecThreads) league_record_kernel(const int32_t* __restrict__ won,
                                                                    const int32_t* __restrict__ draw, int B,
                                                                    float* __restrict__ entry, int count_games) {
    __shared__ int part[kRecThreads / 64][3];
    int w = 0, l = 0, d = 0;
    // the run summary lives in pinned host memory (zero copy): a thread's loads are all issued before the first is
    // used -- one host round trip, where the strided loop waited for each element in turn
    constexpr int PER = 8;
    for (int b0 = threadIdx.x; b0 < B; b0 += PER * kRecThreads) {
        int wa[PER], wb[PER], dv[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int b = b0 + u * kRecThreads;
            wa[u] = b < B ? won[2 * b] : 0;
            wb[u] = b < B ? won[2 * b + 1] : 0;
            dv[u] = b < B ? draw[b] : 0;
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            if (b0 + u * kRecThreads >= B) break;
            const bool w0 = wa[u] != 0, w1 = wb[u] != 0;
            const bool dr = dv[u] != 0 || w0 == w1;
            w += !dr && w0;
            l += !dr && !w0;
            d += dr;
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        w += __shfl_xor(w, m);
        l += __shfl_xor(l, m);
        d += __shfl_xor(d, m);
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        part[wave][0] = w;
        part[wave][1] = l;
        part[wave][2] = d;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int sw = 0, sl = 0, sd = 0;
        for (int k = 0; k < kRecThreads / 64; ++k) {
            sw += part[k][0];
            sl += part[k][1];
            sd += part[k][2];
        }
        // PayoffEntry: GAMES 0, WIN 1, LOSS 2, DRAW 3 (the delta is private to this rank: plain read-modify-write)
        if (count_games) entry[0] += (float)B;
        entry[1] += (float)sw;
        entry[2] += (float)sl;
        entry[3] += (float)sd;
    }
}

}  // namespace

extern "C" int mlg_league_record_runs(const int32_t* won, const int32_t* draw, int32_t B, float* entry,
                                      int32_t count_games, void* stream) {
    MLG_REQUIRE(won && draw && entry, "league_record_runs: null pointer");
    MLG_REQUIRE(B >= 1, "league_record_runs: B=%d", B);
    hipLaunchKernelGGL(league_record_kernel, dim3(1), dim3(kRecThreads), 0, (hipStream_t)stream, won, draw, B, entry,
                       count_games);
    return mlg::check_launch("league_record_runs");
}
