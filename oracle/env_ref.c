/*
 * oracle/env_ref.c -- CPU restatement of the maleague synthetic N-vs-N team battle ("ma" env, spec v1).
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library (as the checker / the timed CPU baseline). The product path never links it.
 *
 * Parity status: the reference's env (maenv.TeamsEnv, external package `maenv @ git+...ma-env.git`,
 * requirements.txt:22, unpinned, absent from the container) cannot be run here, so env arithmetic is
 * PARITY UNPINNED against ma-env. This file restates the build's own frozen spec; the
 * HIP env kernel (ma-league_amd/csrc/env_device.h) is checked bit-exact against it. What IS pinned is
 * the interface the reference consumes (src/steppers/utils/env_worker_process.py:37-60,
 * src/steppers/parallel_stepper.py:168-191): obs/state/avail/reward/done_n/info per step.
 *
 * Spec summary (all integer arithmetic; floats are exact power-of-two scalings of small integers):
 *   units u = 0..U-1 in plan order (team 0 units, then team 1 units); role TANK=0 HEALER=1 ADC=2,
 *   attack RANGED=0 MELEE=1.  max_hp: TANK 64, HEALER 32, ADC 32.  power: TANK 3, HEALER 4 (heal), ADC 6.
 *   range^2: RANGED 9, MELEE 2.  sight^2: 36.
 *   actions: 0 noop (avail iff dead), 1 y+1, 2 y-1, 3 x+1, 4 x-1 (avail iff alive and in bounds),
 *            5+j target unit j: attacker -> enemy j alive in range; healer -> ally j != self alive,
 *            hp_j < max_hp_j, in range.  Dead unit: only noop.  Unavailable chosen action -> noop.
 *   scripted "basic" AI (pre-step state): healer heals lowest-hp damaged ally in range (tie: lowest j),
 *            else moves toward nearest ally (if dist^2 > 2; ties lowest j; no ally alive -> nearest enemy);
 *            attacker attacks lowest-hp enemy in range (tie lowest j), else moves toward nearest enemy.
 *            move toward: |dx| >= |dy| and dx != 0 -> x += sgn(dx); else if dy != 0 -> y += sgn(dy).
 *   resolution: damage/heal from pre-step positions/hp, summed per target; then moves; then
 *            hp' = clamp(hp - dmg + heal, 0, max_hp) for alive units; dead when hp' == 0.
 *   reward(team T) = [sum_{enemy j} max(0, hp_j - hp'_j) + 10*kills + 200*won_T] / 16.
 *   done = a team has no alive units, or t+1 >= episode_limit.  won_T = enemies wiped and T alive.
 *   draw = done and nobody won.
 *   spawns (stochastic): r = rng(key, ctr(episode, 0, SPAWN, u)); team 0 x = r%4, team 1 x = G-1-r%4;
 *            y = (r>>8) % G.  Non-stochastic: x = 1 / G-2, y = (k*G)/n_team + (G/n_team)/2.
 *   obs (agent i, per unit j, 8 features): zero if agent dead or j not visible (dead or dist^2 > 36);
 *            else [1, dx/P, dy/P, hp_j/max_hp_j, avail(i, 5+j), same_team, role_j/2, melee_j],
 *            P = next power of two >= grid_size.
 *   state (per unit j, 6 features): [alive, x/P, y/P, hp/max_hp, team, role/2].
 *   rng(key, ctr) = splitmix64(key ^ splitmix64(ctr)); key = seed * 2^32 + env_index.
 *   ctr(episode, t, purpose, idx) = episode<<32 | t<<16 | purpose<<12 | idx.
 *   purposes: SPAWN=1, EPS=2 (epsilon coin), RAND=3 (random action draw).
 */
#include <stdint.h>
#include <string.h>

#define MAXU 64
#define ACT_BASE 5

static const int ROLE_MAXHP[3] = {64, 32, 32};
static const int ROLE_POWER[3] = {3, 4, 6};
static const int ATK_RANGE2[2] = {9, 2};
static const int SIGHT2 = 36;

uint64_t envref_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

uint64_t envref_rng(uint64_t key, uint64_t ctr) { return envref_splitmix64(key ^ envref_splitmix64(ctr)); }

uint64_t envref_ctr(uint32_t episode, uint32_t t, uint32_t purpose, uint32_t idx) {
    return ((uint64_t)episode << 32) | ((uint64_t)(t & 0xFFFF) << 16) | ((uint64_t)(purpose & 0xF) << 12) |
           (uint64_t)(idx & 0xFFF);
}

float envref_u01(uint64_t r) { return (float)(r >> 40) * (1.0f / 16777216.0f); }

typedef struct {
    int U;             /* total units */
    int n_agents;      /* policy-controlled units */
    int grid;          /* grid_size */
    int episode_limit; /* max steps */
    int stochastic;    /* stochastic spawns */
    int team[MAXU];    /* plan team of unit */
    int role[MAXU];    /* 0 TANK 1 HEALER 2 ADC */
    int melee[MAXU];   /* 0 ranged 1 melee */
    int scripted[2];   /* per plan team */
    int agent_unit[MAXU];
    int team_size[2];
    int team_first[2];
    int policy_team;   /* first non-scripted team */
} envref_spec;

static int pow2_at_least(int g) {
    int p = 1;
    while (p < g) p <<= 1;
    return p;
}

static int dist2(const int *x, const int *y, int i, int j) {
    int dx = x[j] - x[i], dy = y[j] - y[i];
    return dx * dx + dy * dy;
}

int envref_avail_one(const envref_spec *s, const int *x, const int *y, const int *hp, int i, int a) {
    int alive = hp[i] > 0;
    if (a == 0) return !alive;
    if (!alive) return 0;
    if (a == 1) return y[i] + 1 < s->grid;
    if (a == 2) return y[i] - 1 >= 0;
    if (a == 3) return x[i] + 1 < s->grid;
    if (a == 4) return x[i] - 1 >= 0;
    int j = a - ACT_BASE;
    if (j < 0 || j >= s->U) return 0;
    if (hp[j] <= 0) return 0;
    if (dist2(x, y, i, j) > ATK_RANGE2[s->melee[i]]) return 0;
    if (s->role[i] == 1) /* healer */
        return j != i && s->team[j] == s->team[i] && hp[j] < ROLE_MAXHP[s->role[j]];
    return s->team[j] != s->team[i];
}

void envref_reset(const envref_spec *s, uint64_t key, uint32_t episode, int *x, int *y, int *hp) {
    int G = s->grid;
    for (int u = 0; u < s->U; ++u) {
        int tm = s->team[u];
        hp[u] = ROLE_MAXHP[s->role[u]];
        if (s->stochastic) {
            uint64_t r = envref_rng(key, envref_ctr(episode, 0, 1, (uint32_t)u));
            int col = (int)(r % 4u);
            x[u] = tm == 0 ? col : G - 1 - col;
            y[u] = (int)((r >> 8) % (uint64_t)G);
        } else {
            int k = u - s->team_first[tm], n = s->team_size[tm];
            x[u] = tm == 0 ? 1 : G - 2;
            y[u] = (k * G) / n + (G / n) / 2;
        }
    }
}

static void move_toward(const envref_spec *s, const int *x, const int *y, int i, int j, int *act) {
    int dx = x[j] - x[i], dy = y[j] - y[i];
    int adx = dx < 0 ? -dx : dx, ady = dy < 0 ? -dy : dy;
    (void)s;
    if (adx >= ady && dx != 0) *act = dx > 0 ? 3 : 4;
    else if (dy != 0) *act = dy > 0 ? 1 : 2;
    else *act = 0;
}

int envref_ai_action(const envref_spec *s, const int *x, const int *y, const int *hp, int i) {
    if (hp[i] <= 0) return 0;
    int act = 0;
    if (s->role[i] == 1) {
        int best = -1;
        for (int j = 0; j < s->U; ++j)
            if (envref_avail_one(s, x, y, hp, i, ACT_BASE + j) && (best < 0 || hp[j] < hp[best])) best = j;
        if (best >= 0) return ACT_BASE + best;
        int near = -1, nd = 0;
        for (int j = 0; j < s->U; ++j) {
            if (j == i || hp[j] <= 0 || s->team[j] != s->team[i]) continue;
            int d = dist2(x, y, i, j);
            if (near < 0 || d < nd) { near = j; nd = d; }
        }
        if (near >= 0) {
            if (nd > 2) move_toward(s, x, y, i, near, &act);
            return act;
        }
    } else {
        int best = -1;
        for (int j = 0; j < s->U; ++j)
            if (envref_avail_one(s, x, y, hp, i, ACT_BASE + j) && (best < 0 || hp[j] < hp[best])) best = j;
        if (best >= 0) return ACT_BASE + best;
    }
    int near = -1, nd = 0;
    for (int j = 0; j < s->U; ++j) {
        if (hp[j] <= 0 || s->team[j] == s->team[i]) continue;
        int d = dist2(x, y, i, j);
        if (near < 0 || d < nd) { near = j; nd = d; }
    }
    if (near >= 0) move_toward(s, x, y, i, near, &act);
    return act;
}

/*
 * One env step. actions: n_agents policy actions (agent order). t: step index before the step.
 * Outputs: rewards[2] (per plan team, float), done, won[2] (per plan team), draw.
 * x/y/hp updated in place.
 */
void envref_step(const envref_spec *s, int t, const int64_t *actions, int *x, int *y, int *hp, float *rewards,
                 int *done, int *won, int *draw) {
    int U = s->U;
    int act[MAXU], dmg[MAXU], heal[MAXU], hp0[MAXU];
    int is_agent[MAXU];
    memset(is_agent, 0, sizeof(is_agent));
    for (int a = 0; a < s->n_agents; ++a) is_agent[s->agent_unit[a]] = a + 1;
    for (int u = 0; u < U; ++u) {
        if (is_agent[u]) {
            int a = (int)actions[is_agent[u] - 1];
            act[u] = (a >= 0 && a < ACT_BASE + U && envref_avail_one(s, x, y, hp, u, a)) ? a : 0;
        } else {
            act[u] = envref_ai_action(s, x, y, hp, u);
        }
        dmg[u] = 0;
        heal[u] = 0;
        hp0[u] = hp[u];
    }
    for (int i = 0; i < U; ++i) {
        if (hp0[i] <= 0 || act[i] < ACT_BASE) continue;
        int j = act[i] - ACT_BASE;
        if (s->role[i] == 1) heal[j] += ROLE_POWER[1];
        else dmg[j] += ROLE_POWER[s->role[i]];
    }
    for (int i = 0; i < U; ++i) {
        if (hp0[i] <= 0) continue;
        switch (act[i]) {
            case 1: y[i] += 1; break;
            case 2: y[i] -= 1; break;
            case 3: x[i] += 1; break;
            case 4: x[i] -= 1; break;
            default: break;
        }
    }
    int alive[2] = {0, 0}, lost[2] = {0, 0}, kills[2] = {0, 0};
    for (int j = 0; j < U; ++j) {
        if (hp0[j] > 0) {
            int v = hp0[j] - dmg[j] + heal[j];
            int mx = ROLE_MAXHP[s->role[j]];
            v = v < 0 ? 0 : (v > mx ? mx : v);
            hp[j] = v;
            int l = hp0[j] - v;
            lost[s->team[j]] += l > 0 ? l : 0;
            if (v == 0) kills[1 - s->team[j]] += 1;
        }
        if (hp[j] > 0) alive[s->team[j]] += 1;
    }
    int d = alive[0] == 0 || alive[1] == 0 || t + 1 >= s->episode_limit;
    int w0 = alive[1] == 0 && alive[0] > 0, w1 = alive[0] == 0 && alive[1] > 0;
    won[0] = w0;
    won[1] = w1;
    *draw = d && !w0 && !w1;
    *done = d;
    for (int tm = 0; tm < 2; ++tm) {
        int r = lost[1 - tm] + 10 * kills[tm] + 200 * won[tm];
        rewards[tm] = (float)r * 0.0625f;
    }
}

/* obs: [n_agents][8U] */
void envref_obs(const envref_spec *s, const int *x, const int *y, const int *hp, float *obs) {
    int U = s->U;
    float inv_p = 1.0f / (float)pow2_at_least(s->grid);
    memset(obs, 0, sizeof(float) * (size_t)s->n_agents * 8 * U);
    for (int a = 0; a < s->n_agents; ++a) {
        int i = s->agent_unit[a];
        if (hp[i] <= 0) continue;
        for (int j = 0; j < U; ++j) {
            if (hp[j] <= 0 || dist2(x, y, i, j) > SIGHT2) continue;
            float *o = obs + ((size_t)a * U + j) * 8;
            o[0] = 1.0f;
            o[1] = (float)(x[j] - x[i]) * inv_p;
            o[2] = (float)(y[j] - y[i]) * inv_p;
            o[3] = (float)hp[j] * (1.0f / (float)ROLE_MAXHP[s->role[j]]);
            o[4] = (float)envref_avail_one(s, x, y, hp, i, ACT_BASE + j);
            o[5] = (float)(s->team[j] == s->team[i]);
            o[6] = (float)s->role[j] * 0.5f;
            o[7] = (float)s->melee[j];
        }
    }
}

/* state: [6U] */
void envref_state(const envref_spec *s, const int *x, const int *y, const int *hp, float *st) {
    float inv_p = 1.0f / (float)pow2_at_least(s->grid);
    for (int j = 0; j < s->U; ++j) {
        float *o = st + j * 6;
        int al = hp[j] > 0;
        o[0] = (float)al;
        o[1] = (float)x[j] * inv_p;
        o[2] = (float)y[j] * inv_p;
        o[3] = (float)hp[j] * (1.0f / (float)ROLE_MAXHP[s->role[j]]);
        o[4] = (float)s->team[j];
        o[5] = (float)s->role[j] * 0.5f;
    }
}

/* avail: [n_agents][5+U] int32 */
void envref_avail(const envref_spec *s, const int *x, const int *y, const int *hp, int32_t *avail) {
    int A = ACT_BASE + s->U;
    for (int a = 0; a < s->n_agents; ++a)
        for (int k = 0; k < A; ++k) avail[a * A + k] = envref_avail_one(s, x, y, hp, s->agent_unit[a], k);
}

int envref_maxu(void) { return MAXU; }
int envref_sizeof_spec(void) { return (int)sizeof(envref_spec); }

/*
 * Entity variant ("refil" env, config 5). U = 2S units, S slots per team: policy team = units
 * 0..S-1 (they are the agents, entity index = unit index, so entities[:n_agents] are the agents as
 * EntityAttentionRNNAgent assumes, src/marl/modules/agents/entity_rnn_agent.py:38), scripted team = S..2S-1.
 * Per episode k active slots per team, k = kmin + r % (kmax - kmin + 1), r = rng(key, ctr(episode, 0, TEAM=4, 0));
 * absent units have hp 0 for the whole episode (never spawn, never act, never targetable). Everything else is
 * spec v1.
 */
int envref_reset_entity(const envref_spec *s, uint64_t key, uint32_t episode, int kmin, int kmax, int *x, int *y,
                        int *hp) {
    envref_reset(s, key, episode, x, y, hp);
    uint64_t r = envref_rng(key, envref_ctr(episode, 0, 4, 0));
    int k = kmin + (int)(r % (uint64_t)(kmax - kmin + 1));
    for (int u = 0; u < s->U; ++u)
        if (u - s->team_first[s->team[u]] >= k) hp[u] = 0;
    return k;
}

/*
 * Entity observation (the REFIL entity scheme: entities [U][8], obs_mask [U][U], entity_mask [U]; 1 = masked).
 *   entity j (alive): [1, x/P, y/P, hp/max_hp, team, role/2, melee, power/8]; dead or absent: zeros.
 *   entity_mask[j] = hp_j <= 0.   obs_mask[i][j] = hp_i <= 0 || hp_j <= 0 || dist2(i, j) > sight^2.
 */
void envref_entities(const envref_spec *s, const int *x, const int *y, const int *hp, float *ent, uint8_t *obs_mask,
                     uint8_t *entity_mask) {
    int U = s->U;
    float inv_p = 1.0f / (float)pow2_at_least(s->grid);
    for (int j = 0; j < U; ++j) {
        float *o = ent + j * 8;
        entity_mask[j] = hp[j] <= 0;
        if (hp[j] <= 0) {
            for (int f = 0; f < 8; ++f) o[f] = 0.0f;
        } else {
            o[0] = 1.0f;
            o[1] = (float)x[j] * inv_p;
            o[2] = (float)y[j] * inv_p;
            o[3] = (float)hp[j] * (1.0f / (float)ROLE_MAXHP[s->role[j]]);
            o[4] = (float)s->team[j];
            o[5] = (float)s->role[j] * 0.5f;
            o[6] = (float)s->melee[j];
            o[7] = (float)ROLE_POWER[s->role[j]] * 0.125f;
        }
        for (int i = 0; i < U; ++i)
            obs_mask[i * U + j] = hp[i] <= 0 || hp[j] <= 0 || dist2(x, y, i, j) > SIGHT2;
    }
}
