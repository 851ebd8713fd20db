/* Sanitizer driver for the C oracle (TEST INFRASTRUCTURE, SURVEY §5 "Race
 * detection / sanitizers"): `make -C oracle asan ubsan` links vmp_oracle.c
 * with AddressSanitizer / UndefinedBehaviorSanitizer (no recovery) into this
 * program, which walks every exported entry point the tests use:
 *   - reset / step / obs / mask / rank / state / counters over FirstFit,
 *     BestFit and perturbed external actions (invalid targets, suspensions,
 *     negative and out-of-range actions, env.py:35-42) for wr / ut / kl and
 *     the three size sequences, incl. drops (V small against the load) and
 *     reset(seed=None) continuations (env.py:180-226);
 *   - the OpenMP batched rollouts (the CPU baseline of bench.py);
 *   - the scalar-introsort argsort on tie-heavy and NaN keys (bestfit.py:33)
 *     and the numpy RNG known-answer entry points.
 * Exits 0 and prints "oracle sanitize ok" when no sanitizer fired. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../include/vmp.h"

typedef struct oenv oenv;
oenv *oracle_create(const vmp_config *cfg);
void oracle_destroy(oenv *e);
void oracle_reset(oenv *e, int has_seed, int64_t seed);
void oracle_set_eval(oenv *e, int mode);
void oracle_step(oenv *e, const int64_t *action, uint8_t *valid, double *reward, int *terminated);
void oracle_obs(const oenv *e, float *obs);
void oracle_mask(const oenv *e, uint8_t *mask);
void oracle_firstfit(oenv *e, int64_t *action);
void oracle_bestfit(oenv *e, int64_t *action);
int64_t oracle_rank(const oenv *e);
void oracle_get_state(const oenv *e, int64_t *placement, double *vm_cpu, double *vm_mem,
                      double *cpu, double *mem, int64_t *remaining);
void oracle_get_counters(const oenv *e, int64_t *c, double *st);
void oracle_pcg_seed(uint64_t seed, uint64_t out[4]);
void oracle_pcg_raw(uint64_t seed, int64_t n, uint64_t *out);
void oracle_pcg_double(uint64_t seed, int64_t n, double *out);
void oracle_pcg_around(uint64_t seed, int64_t n, double lo, double hi, double *out);
uint64_t oracle_pcg_poisson(uint64_t seed, double lam, int64_t n, int64_t *out);
uint64_t oracle_pcg_advance_raw(uint64_t seed, uint64_t delta);
double oracle_pw_sum(const double *a, int64_t n);
void oracle_argsort_f32(const float *v, int64_t n, int64_t *out);
int64_t oracle_rollout(const vmp_config *cfg, int32_t n_env, int64_t seed0, int64_t stride,
                       int64_t steps, int32_t policy, int32_t eval_mode, int32_t n_threads,
                       double *reward_sum, int64_t *counters);

static uint64_t lcg = 88172645463325252ull;
static uint32_t rnd(void) {
  lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(lcg >> 33);
}

static void run_env(vmp_config c, int steps, int mode) {
  oenv *e = oracle_create(&c);
  const int V = c.vms, P = c.pms, A = c.allow_null_action ? P + 2 : P + 1, D = 3 * V + 2 * P;
  int64_t *act = malloc(sizeof(int64_t) * V), *pl = malloc(sizeof(int64_t) * V);
  int64_t *rem = malloc(sizeof(int64_t) * V), ctr[VMP_NCTR];
  double *vc = malloc(sizeof(double) * V), *vm = malloc(sizeof(double) * V);
  double *cpu = malloc(sizeof(double) * P), *mem = malloc(sizeof(double) * P), st[VMP_NST];
  float *obs = malloc(sizeof(float) * D);
  uint8_t *mask = malloc((size_t)V * A), *valid = malloc(V);
  oracle_set_eval(e, 1);
  for (int t = 0; t < steps; t++) {
    if (mode == 0) oracle_firstfit(e, act);
    else if (mode == 1) oracle_bestfit(e, act);
    else {
      oracle_get_state(e, pl, vc, vm, cpu, mem, rem);
      for (int v = 0; v < V; v++) {
        uint32_t u = rnd() % 100;
        act[v] = pl[v];
        if (u < 10) act[v] = rnd() % A;      /* any target, often invalid */
        else if (u < 13) act[v] = P;          /* suspend (valid if running) */
        else if (u < 14) act[v] = -1 - (int64_t)(rnd() % 3);  /* negative: invalid */
        else if (u < 15) act[v] = A + (rnd() % 5);            /* past NULL: invalid */
      }
    }
    double r;
    int term;
    oracle_step(e, act, valid, &r, &term);
    if (!isfinite(r)) { fprintf(stderr, "non-finite reward\n"); exit(2); }
    oracle_obs(e, obs);
    if (t % 7 == 0) oracle_mask(e, mask);
    (void)oracle_rank(e);
    oracle_get_counters(e, ctr, st);
    if (t == steps / 2) oracle_reset(e, 0, 0);  /* reset(seed=None): streams continue */
  }
  oracle_reset(e, 1, c.seed + 12);
  oracle_destroy(e);
  free(act); free(pl); free(rem); free(vc); free(vm); free(cpu); free(mem);
  free(obs); free(mask); free(valid);
}

int main(void) {
  vmp_config c = {0};
  c.training_steps = 10000;
  c.eval_steps = 100000;
  c.cap_target_util = 1;
  c.allow_null_action = 1;
  c.beta = 0.5;
  const struct { int P, V; double lam, L; int rw, seq, null_ok; } cfgs[] = {
      {10, 30, 0.182, 100, VMP_REWARD_KL, VMP_SEQ_UNIFORM, 1},
      {10, 12, 1.5, 40, VMP_REWARD_WR, VMP_SEQ_HIGHUNIFORM, 1},   /* drops */
      {20, 60, 0.9, 50, VMP_REWARD_UT, VMP_SEQ_LOWUNIFORM, 0},
      {100, 300, 1.8182, 200, VMP_REWARD_KL, VMP_SEQ_UNIFORM, 1},
      {100, 1000, 1.8182, 300, VMP_REWARD_WR, VMP_SEQ_UNIFORM, 1},
      {7, 9, 12.0, 15, VMP_REWARD_KL, VMP_SEQ_UNIFORM, 1},         /* PTRS arrivals */
  };
  for (unsigned i = 0; i < sizeof(cfgs) / sizeof(cfgs[0]); i++) {
    c.pms = cfgs[i].P;
    c.vms = cfgs[i].V;
    c.arrival_rate = cfgs[i].lam;
    c.service_length = cfgs[i].L;
    c.reward_function = cfgs[i].rw;
    c.sequence = cfgs[i].seq;
    c.allow_null_action = cfgs[i].null_ok;
    c.seed = 3 + 4 * i;
    for (int mode = 0; mode < 3; mode++) run_env(c, cfgs[i].V >= 1000 ? 120 : 400, mode);
  }
  /* the OpenMP batched baseline */
  c.pms = 100; c.vms = 300; c.arrival_rate = 1.8182; c.service_length = 100;
  c.reward_function = VMP_REWARD_KL; c.sequence = VMP_SEQ_UNIFORM; c.allow_null_action = 1;
  double rs[8];
  int64_t ctr[8 * VMP_NCTR];
  oracle_rollout(&c, 8, 0, 4, 150, VMP_POLICY_FIRSTFIT, 1, 4, rs, ctr);
  oracle_rollout(&c, 8, 0, 4, 150, VMP_POLICY_BESTFIT, 0, 4, rs, ctr);
  /* argsort: ties, NaN, sizes across the insertion / quicksort / heapsort paths */
  for (int n = 0; n <= 1500; n += (n < 40 ? 1 : 97)) {
    float *v = malloc(sizeof(float) * (n + 1));
    int64_t *o = malloc(sizeof(int64_t) * (n + 1));
    for (int k = 0; k < n; k++) v[k] = (float)(rnd() % 7) * 0.25f;
    if (n > 5) v[n / 2] = NAN;
    oracle_argsort_f32(v, n, o);
    for (int k = 1; k < n; k++)
      if (v[o[k]] < v[o[k - 1]]) { fprintf(stderr, "argsort order\n"); return 3; }
    free(v);
    free(o);
  }
  /* numpy RNG entry points */
  uint64_t s4[4], raw[64];
  double d[64];
  int64_t pz[64];
  oracle_pcg_seed(0xdeadbeafull, s4);
  oracle_pcg_raw(5, 64, raw);
  oracle_pcg_double(6, 64, d);
  oracle_pcg_around(7, 64, 0.1, 1.0, d);
  const double lams[] = {0.0, 0.0182, 0.182, 1.8182, 9.99, 10.0, 100.0, 1000.0, 4100.0};
  for (unsigned i = 0; i < sizeof(lams) / sizeof(lams[0]); i++) oracle_pcg_poisson(8, lams[i], 64, pz);
  (void)oracle_pcg_advance_raw(9, 1ull << 40);
  (void)oracle_pw_sum(d, 64);
  printf("oracle sanitize ok\n");
  return 0;
}
