/*
 * vmp.h — C ABI of libvmp.so, the MI355X-native batched VM placement/migration
 * environment (drop-in for the reference's `VmEnv` gym plugin path).
 *
 * The reference boundary is a Python gymnasium plugin, not an FFI:
 *   register("VmEnv-v1", entry_point="vmenv.envs.env:VmEnv")   vmenv/__init__.py:3-6
 *   env = gym.make("VmEnv-v1", config=Config(**env_cfg))        main.py:47
 * Every entry point below replaces one method of that class (or of the
 * FirstFit/BestFit agents) for N independent env instances at once; the
 * Python layer (vmp/env.py, vmp/batched.py) binds them with ctypes and keeps
 * the reference's reset()/step()/get_invalid_action_mask() surface.
 *
 * Conventions
 *  - All array pointers passed to a handle created on a GPU are DEVICE
 *    pointers (e.g. torch.Tensor.data_ptr() on that device); sizes are in
 *    elements. Layouts are env-major: x[env][...].
 *  - Every call returns 0 on success or a negative VMP_E* code; the message of
 *    the last failure on this thread is vmp_last_error().
 *  - Invalid actions are never errors: they are no-ops reported in `valid`
 *    (env.py:71-72).
 *  - A handle is bound to one HIP stream (vmp_set_stream) and is not
 *    thread-safe; different handles may be used from different threads.
 */
#ifndef VMP_H
#define VMP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VMP_ABI_VERSION 11

#define VMP_OK 0
#define VMP_EINVAL (-1)
#define VMP_EDEVICE (-2)
#define VMP_EOOM (-3)
#define VMP_ESTATE (-4)

/* reward_function (env.py:123-156) */
#define VMP_REWARD_WR 0
#define VMP_REWARD_UT 1
#define VMP_REWARD_KL 2
/* sequence (env.py:211-219) */
#define VMP_SEQ_UNIFORM 0
#define VMP_SEQ_LOWUNIFORM 1
#define VMP_SEQ_HIGHUNIFORM 2
/* eval-mode Record metrics (vmp_record_read): per-env sums, VMP_NREC doubles */
#define VMP_REC_STEPS 0     /* recorded steps */
#define VMP_REC_REWARD 1    /* sum of rewards */
#define VMP_REC_CPU 2       /* sum over steps and PMs of cpu, and of cpu^2 */
#define VMP_REC_CPU2 3
#define VMP_REC_MEM 4       /* same for memory */
#define VMP_REC_MEM2 5
#define VMP_REC_RANK 6      /* sum of _get_rank (PMs hosting >= 1 VM) */
#define VMP_REC_DROP 7      /* sum of dropped / total_requests (0 if none) */
#define VMP_REC_TCM 8       /* sum of target_cpu_mean, target_memory_mean */
#define VMP_REC_TMM 9
#define VMP_REC_WAITING 10  /* sum of waiting_ratio */
#define VMP_REC_LIFE_SUM 11 /* sum of VM lifetimes (record.py vm_lifetime) */
#define VMP_REC_LIVES 12    /* number of VM lives (len(unique_vms_placement)) */
#define VMP_REC_REWARD_OK 13 /* sum and count of rewards > -1e7, count of rewards < -1e7 */
#define VMP_REC_N_OK 14
#define VMP_REC_N_BAD 15
#define VMP_REC_CPUVAR 16   /* sum over steps of var over PMs of cpu, of memory */
#define VMP_REC_MEMVAR 17   /*   (exp_performance.py:109-113, exp_vm_size.py:78-83) */
#define VMP_REC_XMEM 18     /* sum over steps and PMs of mem[e][p] * sum_s mem[s][p] over the
                               handle's envs: their sum over e is the cross-env square
                               exp_performance.py:114 (np.var(memory, axis=0)) needs; 0 when
                               n_env > VMP_REC_XMAX */
#define VMP_NREC 19
#define VMP_REC_XMAX 64
#define VMP_REC_BINS 1001   /* pending / slowdown rates x1000: 0 .. 1000 */
/* actor-head modes (vmp_policy_head) */
#define VMP_HEAD_SAMPLE 0 /* Network.get_action(obs, action=None, mask) (ppo.py:115-126) */
#define VMP_HEAD_GIVEN 1  /* Network.get_action(obs, action, mask): log_prob/entropy only */
#define VMP_HEAD_ARGMAX 2 /* Network.get_det_action (ppo.py:128-131): unmasked argmax */
#define VMP_HEAD_MAX_A 1024 /* action_dim limit of the register-resident row */
#define VMP_ACTOR_HEAD_MAX_A 128 /* action_dim limit of the fused GEMM + head (vmp_actor_head) */
/* heuristic policies (src/agents/firstfit.py:21-38, bestfit.py:21-40) */
#define VMP_POLICY_FIRSTFIT 0
#define VMP_POLICY_BESTFIT 1

/* Mirrors vmenv/envs/config.py:4-15 field for field. */
typedef struct vmp_config {
  double arrival_rate;      /* Poisson lambda per step */
  double service_length;    /* Poisson mean; runtime = poisson(L) + 1 */
  int32_t pms;              /* P */
  int32_t vms;              /* V (slots) */
  int64_t training_steps;
  int64_t eval_steps;
  int64_t seed;
  int32_t reward_function;  /* VMP_REWARD_* */
  int32_t sequence;         /* VMP_SEQ_* */
  int32_t cap_target_util;  /* bool */
  int32_t allow_null_action;/* bool: A = P+2 if true else P+1 (env.py:26) */
  double beta;
} vmp_config;

/* Per-env counters, vmp_get_counters() row layout (env.py:196-205, 299-318). */
#define VMP_CTR_TOTAL_REQUESTS 0
#define VMP_CTR_SERVED 1
#define VMP_CTR_SUSPEND 2
#define VMP_CTR_PLACE 3
#define VMP_CTR_DROPPED 4
#define VMP_CTR_TIMESTEP 5
#define VMP_NCTR 6
/* Per-env float stats, vmp_get_stats() row layout. */
#define VMP_ST_WAITING_RATIO 0
#define VMP_ST_TARGET_CPU_MEAN 1
#define VMP_ST_TARGET_MEM_MEAN 2
#define VMP_ST_TOTAL_CPU_REQ 3
#define VMP_ST_TOTAL_MEM_REQ 4
#define VMP_NST 5

typedef struct vmp_handle vmp_handle;

int vmp_abi_version(void);
const char *vmp_last_error(void);

/* VmEnv.__init__ (env.py:23-33) for n_env instances on HIP device `device`.
 * Every env is reset with seeds[i] (host array, n_env entries), i.e.
 * reset(seed=seeds[i]) -> four numpy PCG64 streams seeded seeds[i]+k
 * (env.py:172-178). eval_mode starts false (env.py:25). */
int vmp_create(const vmp_config *cfg, int32_t n_env, const int64_t *seeds, int32_t device,
               vmp_handle **out);
int vmp_destroy(vmp_handle *h);
int vmp_set_stream(vmp_handle *h, void *hip_stream);
/* VmEnv.eval (env.py:105-106). */
int vmp_set_eval(vmp_handle *h, int32_t eval_mode);
/* Shape helpers: A = action_dim (env.py:26), D = obs dim (env.py:27). */
int vmp_dims(const vmp_handle *h, int32_t *n_env, int32_t *P, int32_t *V, int32_t *A,
             int32_t *D);

/* VmEnv.reset (env.py:180-226) for the envs whose env_mask byte is non-zero
 * (env_mask may be NULL = all). seeds: device int64[n_env] or NULL; a NULL
 * seeds array is reset(seed=None): streams continue and the VM-size
 * sequences restart 2*max(training_steps, eval_steps) draws further
 * (env.py:181-182, 211-219). obs (nullable): device f32[n_env][D]. */
int vmp_reset(vmp_handle *h, const int64_t *seeds, const uint8_t *env_mask, float *obs);

/* VmEnv.step (env.py:66-103) for every env.
 *  actions: device int32[n_env][V]
 *  obs:     device f32[n_env][D]  (nullable)     env.py:295-296
 *  reward:  device f64[n_env]     (nullable)     env.py:123-156
 *  done:    device u8[n_env]      (nullable)     env.py:160-163
 *  valid:   device u8[n_env][V]   (nullable)     env.py:68-72 */
int vmp_step(vmp_handle *h, const int32_t *actions, float *obs, double *reward,
             uint8_t *done, uint8_t *valid);
/* vmp_step that also writes the invalid-action mask of the state it leaves
 * (get_invalid_action_mask, env.py:45-53, as vmp_mask lays it out) into
 * next_mask_bits (nullable): the mask the next PPOAgent.act reads
 * (ppo.py:151-153), without a separate vmp_mask launch per step. (ABI 11) */
int vmp_step_mask(vmp_handle *h, const int32_t *actions, float *obs, double *reward,
                  uint8_t *done, uint8_t *valid, uint32_t *next_mask_bits);

/* FirstFitAgent.act / BestFitAgent.act (firstfit.py:21-38, bestfit.py:21-40)
 * on the current observation of every env -> device int32[n_env][V]. */
int vmp_heuristic_act(vmp_handle *h, int32_t policy, int32_t *actions);

/* The same agents on a CALLER's observation, device f32[n_env][3V+2P]
 * (firstfit.py:21-38 / bestfit.py:21-40 read only the obs they are passed,
 * utils.py:37-47): f32 fit tests on the obs values, FirstFit updating cpu
 * only, BestFit in flip(argsort(cpu+memory)) order with numpy's scalar
 * introsort ties; no env state is read. -> device int32[n_env][V]. P <= 3583. */
int vmp_heuristic_act_obs(vmp_handle *h, int32_t policy, const float *obs, int32_t *actions);

/* act + step fused in one launch: the action the heuristic takes on the
 * pre-step observation is applied by step() in the same kernel (the
 * Base.test loop body, base.py:71-86). actions_out (nullable) receives it. */
int vmp_heuristic_step(vmp_handle *h, int32_t policy, int32_t *actions_out, float *obs,
                       double *reward, uint8_t *done, uint8_t *valid);

/* K fused heuristic steps per env in one launch, state resident on chip.
 * rewards: device f64[k_steps][n_env] (nullable); done_count: device
 * int64[n_env] (nullable) accumulates the steps whose `terminated` was true. */
int vmp_rollout_heuristic(vmp_handle *h, int32_t policy, int32_t k_steps, double *rewards,
                          int64_t *done_count);

/* VmEnv.get_invalid_action_mask(masked=True) (env.py:45-53), bit-packed:
 * device u32[n_env][V][W], W = ceil(A/32); bit a of row v set = invalid. */
int vmp_mask(vmp_handle *h, uint32_t *bits);
/* Same mask expanded to the reference's bool layout: device u8[n_env][V][A]. */
int vmp_mask_bool(vmp_handle *h, uint8_t *mask);

/* Observation of the current state (env.py:295-296): device f32[n_env][D]. */
int vmp_get_obs(vmp_handle *h, float *obs);
/* Counters (VMP_CTR_*): device int64[n_env][VMP_NCTR]. */
int vmp_get_counters(vmp_handle *h, int64_t *counters);
/* Stats (VMP_ST_*): device f64[n_env][VMP_NST]. */
int vmp_get_stats(vmp_handle *h, double *stats);
/* Full reference-dtype state (info / parity): device arrays, each nullable.
 * placement, remaining: int64[n_env][V]; vm_cpu, vm_mem: f64[n_env][V];
 * cpu, mem: f64[n_env][P]. */
int vmp_get_state(vmp_handle *h, int64_t *placement, double *vm_cpu, double *vm_mem,
                  double *cpu, double *mem, int64_t *remaining);
/* _get_rank (env.py:320-325) = number of PMs hosting >= 1 VM: int64[n_env]. */
int vmp_get_rank(vmp_handle *h, int64_t *rank);

/* Checkpoint / resume of the batched env state (the reference only
 * saves the policy weights, ppo.py:163-170). vmp_snapshot copies everything a
 * later reset/step reads — the four PCG64 streams and sequence bases, counters,
 * step hints, PM resources and VM words with their finish keys — into a
 * device buffer of vmp_snapshot_bytes() bytes (16-byte aligned); vmp_restore
 * writes it into a handle of the same env count and config (the config's seed
 * field may differ), which then continues bit-exactly where the snapshotted
 * handle stood. Stream-ordered on the handle's stream (vmp_snapshot returns
 * after the copy; vmp_restore synchronises the stream once to check the
 * snapshot's descriptor). Not included: eval mode (vmp_set_eval) and the
 * Record recorder (re-enable it after a restore, as after a reset). */
int vmp_snapshot_bytes(const vmp_handle *h, int64_t *bytes);
int vmp_snapshot(vmp_handle *h, void *dst);
int vmp_restore(vmp_handle *h, const void *src);

/* PPOAgent.update GAE (ppo.py:232-243) over T steps x N envs, reverse scan:
 *  delta = r + (1-d)*gamma*v' - v;  g = delta + (1-d)*gamma*lambda*g.
 * All device f32 [T][N] (done as f32 0/1); adv and ret are outputs. */
int vmp_gae(int32_t T, int32_t N, const float *reward, const float *done, const float *value,
            const float *next_value, float gamma, float lam, float *adv, float *ret,
            void *hip_stream);

/* Network.get_action head (ppo.py:115-126) on the actor's logits f32[B][V*A]
 * (row-major, as nn.Linear writes them): rows flagged in mask_bits u32[B][V][W]
 * (W = ceil(A/32), nullable = get_action(..., invalid_mask=None)) are set to
 * -1e7 as ppo.py:119 does, then per (b, v) a Categorical over A.
 *  - VMP_HEAD_SAMPLE: action[b][v] drawn (inverse CDF, counter-based uniforms
 *    from (seed, offset + b*V + v)); VMP_HEAD_GIVEN: action read.
 *    logprob[b] = sum_v log p(action), entropy[b] = sum_v H (ppo.py:123-126),
 *    both nullable.
 *  - VMP_HEAD_ARGMAX: get_det_action (ppo.py:128-131), argmax of the unmasked
 *    row, first index on ties; logprob/entropy untouched.
 *  - rng_counter (nullable): a device u64 whose current value is mixed into the
 *    seed, so a captured graph that advances it between replays draws fresh
 *    actions; workspace (nullable): 2*B*V floats of row scratch (else the call
 *    allocates stream-ordered memory, which graph capture may not support).
 *  - wait_ratio >= 0 applies PPOAgent.act's WAIT coin flips first (ppo.py:154-156):
 *    a row with > 1 invalid entries whose column wait_index (= P) is valid
 *    gets it forbidden when a uniform draw exceeds wait_ratio
 *    (migration_ratio). wait_ratio < 0: no flips (PPOAgent.learn, ppo.py:197).
 * Replaces the torch Categorical / multinomial calls of ppo.py:117-126.
 * All pointers are device pointers; A <= VMP_HEAD_MAX_A. */
int vmp_policy_head(int32_t B, int32_t V, int32_t A, int32_t mode, const float *logits,
                    const uint32_t *mask_bits, float wait_ratio, int32_t wait_index,
                    uint64_t seed, uint64_t offset, const uint64_t *rng_counter, int32_t *action,
                    float *logprob, float *entropy, float *workspace, void *hip_stream);

/* Backward of vmp_policy_head (VMP_HEAD_SAMPLE/GIVEN, no coin flips) for the
 * PPO loss (ppo.py:258-277): given dL/dlogprob[B] and dL/dentropy[B]
 * (nullable = 0), writes dL/dlogits f32[B][V*A]; masked entries get 0 (the
 * in-place mask assignment of ppo.py:119 passes no gradient). dlogits may
 * alias logits (the rows are read before they are written). */
int vmp_policy_head_backward(int32_t B, int32_t V, int32_t A, const float *logits,
                             const uint32_t *mask_bits, const int32_t *action,
                             const float *g_logprob, const float *g_entropy, float *dlogits,
                             void *hip_stream);

/* vmp_policy_head_backward with bf16 dlogits (round to nearest even), for the
 * bf16-GEMM training leg whose dW / dh GEMMs take bf16 inputs: the cast pass
 * over the [B, V*A] gradient is folded into the head's store. Tiled path only:
 * A <= 128, logits 16-byte and dlogits 8-byte aligned; dlogits must not alias
 * logits. Not a parity path (the reference trains in f32). */
int vmp_policy_head_backward_bf16(int32_t B, int32_t V, int32_t A, const float *logits,
                                  const uint32_t *mask_bits, const int32_t *action,
                                  const float *g_logprob, const float *g_entropy,
                                  uint16_t *dlogits_bf16, void *hip_stream);

/* The actor's last Linear fused with the head above (ppo.py:115-131, SURVEY
 * §8(f)1): logits = h W^T + bias (h f32[B][K], weight f32[V*A][K] as nn.Linear
 * stores it, bias f32[V*A]) computed on the f32 matrix cores and consumed by
 * the head inside the same workgroup, so the [B, V*A] logits are never written
 * unless logits_out (nullable, f32[B][V*A]) asks for them (the training
 * forward keeps them for vmp_policy_head_backward). Modes, mask, coin flips,
 * rng and outputs as vmp_policy_head (the same per-row uniforms: equal logits
 * draw equal actions). Needs K % 32 == 0, A <= VMP_ACTOR_HEAD_MAX_A and
 * 16-byte aligned h / weight. */
int vmp_actor_head(int32_t B, int32_t K, int32_t V, int32_t A, int32_t mode, const float *h,
                   const float *weight, const float *bias, const uint32_t *mask_bits,
                   float wait_ratio, int32_t wait_index, uint64_t seed, uint64_t offset,
                   const uint64_t *rng_counter, int32_t *action, float *logprob, float *entropy,
                   float *logits_out, float *workspace, void *hip_stream);

/* The actor MLP forward (ppo.py:98-109: Linear(D, H), Tanh, Linear(H, H),
 * Tanh, Linear(H, N)) in f32 for rollouts and eval, one launch: x f32[B][D]
 * (the observations), b1, b2 f32[H] and b3 f32[N] the biases, `packed` the
 * three weight matrices (nn.Linear's w1 f32[H][D], w2 f32[H][H], w3 f32[N][H])
 * in the kernel's MFMA-fragment order, written by vmp_actor_mlp_pack into
 * vmp_actor_mlp_packed_floats(D, H, N, layers) floats (16-byte aligned); the
 * caller re-packs whenever a weight changes. layers = 3: out = the logits
 * f32[B][N]; layers = 2: out = self.actor[:-1](x), the last hidden layer
 * after its Tanh, f32[B][H] (the big heads of config/100.yml go on to
 * vmp_actor_head; w3 / b3 unused). 16 rows per workgroup on the f32 matrix
 * cores, activations kept in LDS between layers. Needs H % 32 == 0, H <= 512,
 * N <= 512, D <= VMP_ACTOR_MLP_MAX_D. Forward only (no autograd). (ABI 11) */
#define VMP_ACTOR_MLP_MAX_D 1536
int64_t vmp_actor_mlp_packed_floats(int32_t D, int32_t H, int32_t N, int32_t layers);
int vmp_actor_mlp_pack(int32_t D, int32_t H, int32_t N, int32_t layers, const float *w1,
                       const float *w2, const float *w3, float *packed, void *hip_stream);
int vmp_actor_mlp_f32(int32_t B, int32_t D, int32_t H, int32_t N, int32_t layers, const float *x,
                      const float *packed, const float *b1, const float *b2, const float *b3,
                      float *out, void *hip_stream);
/* The same MLP with the masked head of vmp_policy_head on its logits in one
 * launch (ppo.py:98-131 Network.get_action / get_det_action with the
 * PPOAgent.act WAIT coin, ppo.py:151-156): N = V * A <= 512, A <= 128; modes,
 * mask bits, coin, rng stream and outputs exactly as vmp_policy_head (the
 * per-row code is shared, so equal logits draw equal actions and give equal
 * logprob / entropy, bit for bit); logits_out (nullable, f32[B][V*A]) keeps a
 * copy of the logits. The logits otherwise never leave the workgroup: one
 * launch per batched step of the eval loop (base.py:71-86). advance_counter
 * (with rng_counter u64[2]): the launch itself adds 1 to rng_counter[0] once
 * every workgroup has read it (rng_counter[1] is the arrival ticket, 0
 * between launches), instead of a separate increment launch. (ABI 11) */
int vmp_actor_mlp_head_f32(int32_t B, int32_t D, int32_t H, int32_t V, int32_t A, int32_t mode,
                           const float *x, const float *packed, const float *b1, const float *b2,
                           const float *b3, const uint32_t *mask_bits, float wait_ratio,
                           int32_t wait_index, uint64_t seed, uint64_t offset,
                           const uint64_t *rng_counter, int32_t advance_counter,
                           int32_t *action, float *logprob, float *entropy, float *logits_out,
                           void *hip_stream);

/* Training side of the fused actor head in bf16: the update's
 * get_action(obs, action, mask) (ppo.py:115-126, called at ppo.py:258) and its
 * backward, for the bf16 training leg (not the parity path: the reference
 * trains in f32). h bf16[B][K] (the actor's last hidden layer rounded to
 * bf16), weight bf16[V*A][K], bias f32[V*A], mask_bits as vmp_policy_head
 * (nullable), action i32[B][V] (GIVEN). Needs K % 64 == 0, A <= 128, 16-byte
 * aligned h / weight / mask_bits (a row's mask words are read as one vector)
 * and, for the backward, 4-byte aligned dlogits (stored as bf16 pairs).
 * Forward: logprob / entropy f32[B] of the given actions; logits formed tile
 * by tile on the bf16 matrix cores (f32 accumulate) and consumed in
 * registers, never written. workspace: nullable, 2*B*V floats. */
int vmp_actor_head_bf16_fwd(int32_t B, int32_t K, int32_t V, int32_t A, const uint16_t *h,
                            const uint16_t *weight, const float *bias, const uint32_t *mask_bits,
                            const int32_t *action, float *logprob, float *entropy,
                            float *workspace, void *hip_stream);
/* Rollout sampling on the same kernel (the bf16 leg's collect: get_action(obs,
 * mask) ppo.py:115-126 and PPOAgent.act's WAIT coin ppo.py:151-156, as
 * vmp_policy_head / vmp_actor_head in VMP_HEAD_SAMPLE mode): action
 * i32[B][V] is the OUTPUT, drawn per (sample, VM row) by inverse CDF over
 * the masked softmax in action order with the counter-based uniform of
 * vmp_policy_head's stream (seed, offset + b*V + v; rng_counter nullable,
 * mixed into the seed as there); wait_ratio >= 0 applies the WAIT coin at
 * column wait_index (needs mask_bits). logprob / entropy f32[B] of the drawn
 * actions. The logits never reach memory. (ABI 10) */
int vmp_actor_head_bf16_sample(int32_t B, int32_t K, int32_t V, int32_t A, const uint16_t *h,
                               const uint16_t *weight, const float *bias,
                               const uint32_t *mask_bits, float wait_ratio, int32_t wait_index,
                               uint64_t seed, uint64_t offset, const uint64_t *rng_counter,
                               int32_t *action, float *logprob, float *entropy, float *workspace,
                               void *hip_stream);
/* Backward: recomputes the logits tiles and writes
 *   dlogits[b][ld] = bf16(d logprob/entropy loss / d logits)  (ld >= V*A)
 * with g_logprob / g_entropy f32[B] (nullable: 0), masked entries 0, as
 * vmp_policy_head_backward_bf16 computes from stored logits. The caller runs
 * it over row chunks (pointers offset to the chunk) and feeds each chunk's
 * dlogits to the dW / dh GEMMs, so no [B, V*A] tensor is ever allocated.
 * dbias (nullable): f32[V*A], ADDED to: the bias gradient of the chunk, the
 * column sums of its dlogits in f32 before the bf16 rounding, formed inside
 * the kernel (per-wave sums in LDS, one partial per M group, reduced in a
 * fixed order: run-to-run identical), so no pass over the dlogits computes
 * it. workspace (nullable): vmp_actor_head_bf16_bwd_workspace(B, V, A) floats
 * for the partials (else stream-ordered memory is allocated). */
int vmp_actor_head_bf16_bwd(int32_t B, int32_t K, int32_t V, int32_t A, const uint16_t *h,
                            const uint16_t *weight, const float *bias, const uint32_t *mask_bits,
                            const int32_t *action, const float *g_logprob,
                            const float *g_entropy, uint16_t *dlogits, int32_t ld, float *dbias,
                            float *workspace, void *hip_stream);
int64_t vmp_actor_head_bf16_bwd_workspace(int32_t B, int32_t V, int32_t A);

/* Eval-mode Record metrics on the device (record.py:34-134, base.py:131-148):
 * on = 1 allocates the recorder and starts it from the current state (call it
 * right after reset, as Base.test records from reset); every later vmp_step /
 * vmp_heuristic_step / vmp_rollout_heuristic step is recorded for every env.
 * on = 0 frees it. */
int vmp_record_enable(vmp_handle *h, int32_t on);
/* Read the metrics so far (non-destructive): hist u32[n_env][2][VMP_REC_BINS]
 * = counts of the pending and slowdown rates rounded to 3 decimals (x1000),
 * over every VM life incl. the open ones; sums f64[n_env][VMP_NREC]. The
 * Record.get_summary values follow from these (vmp/record.py). */
int vmp_record_read(vmp_handle *h, uint32_t *hist, double *sums);

/* Fault injection (tests only): the n-th device allocation made by the
 * library from now on fails as out of memory (n = 0: off). Drives the
 * failure and cleanup paths of vmp_create / vmp_record_enable / vmp_mask_bool
 * under the host sanitizers (tests/native/capi_faults.cpp). */
int vmp_debug_fail_alloc(int32_t n);
/* Number of device allocations the library currently holds (all handles):
 * back to its previous value after a failed call or a vmp_destroy. */
int64_t vmp_debug_live_allocs(void);

/* Diagnostics: per-env shader-clock cycles per kernel phase, accumulated since
 * the previous call, device u64[n_env][24] (see tools/stamps.py for the phase names).
 * Only a library built with -DVMP_STAMPS records them; otherwise
 * returns VMP_EINVAL. */
int vmp_debug_stamps(vmp_handle *h, uint64_t *out);

/* Diagnostics (-DVMP_CHECK_QUIET check build, `make check-quiet`): the number
 * of per-step launches, since the previous call, that skipped the heuristic
 * on the header's quiet bit (EnvHdr::pad bit 62) although some pending VM
 * fitted a PM — always 0 unless an entry point that writes env state left the
 * bit stale. The check build evaluates the fit test on quiet steps too.
 * Returns VMP_EINVAL in a normal build. */
int vmp_debug_quiet_violations(int64_t *count);

/* Diagnostics: workgroups per CU the runtime reports for the per-step env
 * kernel of this handle (hipOccupancyMaxActiveBlocksPerMultiprocessor) and
 * the LDS bytes it is launched with (dynamic + static). */
int vmp_debug_occupancy(vmp_handle *h, int32_t *blocks_per_cu, int32_t *lds_bytes);

#ifdef __cplusplus
}
#endif
#endif /* VMP_H */
