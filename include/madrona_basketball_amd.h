/*
 * madrona_basketball_amd.h -- C ABI of the MI355X-native batched basketball
 * simulator (the drop-in boundary for the reference's step path).
 *
 * Each entry point replaces one piece of the reference's Manager / nanobind
 * surface (davidj24/madrona_basketball):
 *
 *   bb_create / bb_create_with_buffers
 *       <- Manager::Manager(Config, GridState)        src/mgr.cpp:236-239
 *          + the binding's ctor                        src/bindings.cpp:18-61
 *   bb_destroy          <- Manager::~Manager           src/mgr.cpp:241
 *   bb_step             <- Manager::step               src/mgr.cpp:243-246
 *   bb_step_n           <- n x Manager::step (+ optional on-device random
 *                          actions, the bench workload of scripts/run.py:6-19)
 *   bb_step_n_staged    <- n x (actions[:] = a_k; Manager::step), the
 *                          scripts/run.py:10-15 loop with a_k staged in HBM
 *   bb_fill_random_actions <- (new) stages a_k for bb_step_n_staged
 *   bb_rollout          <- n x (actions[:] = a_k; Manager::step; copy of
 *                          observations/rewards/dones), the rollout loop of
 *                          scripts/ppo.py:61-141 with a_k staged in HBM
 *   bb_record           <- the per-step trajectory logging of scripts/ppo.py:93-106
 *                          and scripts/infer.py:116-129 (ten .cpu() copies per
 *                          step), as one device-side copy into a ring
 *   bb_policy_forward   <- Agent.forward of scripts/agent.py:140-154 (32 channels,
 *                          2 layers, env.py:107) + the action write of
 *                          scripts/env.py:147, fused on the device
 *   bb_rollout_policy   <- rollout() of scripts/ppo.py:61-141: n x (agent(obs);
 *                          env.step; buffer stores) + agent.evaluate(obs_)
 *   bb_set_action       <- Manager::setAction          src/mgr.cpp:270-293
 *   bb_trigger_reset    <- Manager::triggerReset       src/mgr.cpp:297-311
 *   bb_export           <- Manager::*Tensor() getters  src/mgr.cpp:317-445
 *                          (exportTensor, src/mgr.cpp:74-80, 121-126)
 *   bb_buffer_bytes     <- (new) sizes for caller-owned storage
 *   bb_last_error       <- (new) the reference aborts via FATAL/REQ_CUDA
 *                          (src/mgr.cpp:191,198) or printf (:289-292);
 *                          this ABI returns status codes instead.
 *
 * Plain C types only.  All device pointers are HIP device pointers on the
 * simulator's gpu_id; `stream` is a hipStream_t passed as void* (NULL = the
 * default stream).  No function aborts; every function returns BB_OK or a
 * negative error code and records a message for bb_last_error().
 */
#ifndef MADRONA_BASKETBALL_AMD_H
#define MADRONA_BASKETBALL_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BB_ABI_VERSION 1

/* status codes */
#define BB_OK 0
#define BB_ERR_INVALID_ARG (-1)
#define BB_ERR_UNSUPPORTED (-2)
#define BB_ERR_HIP (-3)
#define BB_ERR_OOM (-4)

/* madrona::ExecMode (madrona_basketball.madrona.ExecMode) */
#define BB_EXEC_CPU 0
#define BB_EXEC_CUDA 1   /* the HIP/gfx950 path; named as in the reference */

/* dtypes reported by bb_export (madrona::py::TensorElementType subset) */
#define BB_DTYPE_INT32 0
#define BB_DTYPE_FLOAT32 1

/* config flags */
#define BB_FLAG_PER_WORLD_RNG 0x1u /* key each world's RNG by its global index
                                      (reference: every world shares key
                                      split_i(initKey(0),0,0), src/sim.cpp:89) */
#define BB_FLAG_NO_TAG_MASK   0x2u /* drop the tag override of game.cpp:526-528 */
#define BB_FLAG_FULL_GAME     0x4u /* isOneOnOne = 0 (constants.hpp:27 = 0) */

/* Export ids: exactly src/types.hpp:10-42, then build-internal state. */
#define BB_EXPORT_RESET 0
#define BB_EXPORT_GAME_STATE 1
#define BB_EXPORT_ACTION 2
#define BB_EXPORT_ACTION_MASK 3
#define BB_EXPORT_AGENT_POS 4
#define BB_EXPORT_OBSERVATIONS 5
#define BB_EXPORT_REWARD 6
#define BB_EXPORT_DONE 7
#define BB_EXPORT_AGENT_ENTITY_ID 8
#define BB_EXPORT_AGENT_POSSESSION 9
#define BB_EXPORT_ORIENTATION 10
#define BB_EXPORT_TEAM 11
#define BB_EXPORT_AGENT_STATS 12
#define BB_EXPORT_BALL_POS 13
#define BB_EXPORT_BALL_PHYSICS 14
#define BB_EXPORT_BALL_ENTITY_ID 15
#define BB_EXPORT_BALL_GRABBED 16
#define BB_EXPORT_BALL_VELOCITY 17
#define BB_EXPORT_HOOP_POS 18
#define BB_NUM_REFERENCE_EXPORTS 19
#define BB_INTERNAL_AGENT_VELOCITY 32
#define BB_INTERNAL_GRAB_COOLDOWN 33
#define BB_INTERNAL_CUR_STEP 34
#define BB_INTERNAL_INBOUNDING 35
#define BB_INTERNAL_ATTRIBUTES 36
#define BB_INTERNAL_WORLD_CLOCK 37
#define BB_INTERNAL_RNG_COUNTER 38
#define BB_INTERNAL_FIRST 32
#define BB_INTERNAL_LAST 38

typedef struct bb_sim bb_sim;

typedef struct bb_config {
    int64_t discrete_x;          /* grid cells, cellsPerMeter = 1 (bindings.cpp:29-33) */
    int64_t discrete_y;
    float start_x;               /* GridState.startX/Y (ball start, spawn centre) */
    float start_y;
    int64_t max_episode_length;  /* accepted and ignored, as in the reference */
    int32_t exec_mode;           /* BB_EXEC_CPU or BB_EXEC_CUDA */
    int32_t gpu_id;              /* -1: current device */
    int64_t num_worlds;          /* worlds owned by this simulator (this rank's shard) */
    int64_t world_offset;        /* global index of local world 0 (sharding) */
    uint32_t rand_seed;          /* reference hard-codes 0 (bindings.cpp:37) */
    uint32_t flags;              /* BB_FLAG_* */
    int32_t num_agents;          /* 2 = the reference game; 4 and 10 = extensions */
    int32_t reserved;
} bb_config;

/* Fill *cfg with the reference defaults (scripts/env.py:20-35 constructor). */
int bb_default_config(bb_config *cfg);

/* Observation row width for num_agents (128 at 2 agents, src/types.hpp:166). */
int32_t bb_obs_width(int32_t num_agents);

/* Bytes of buffer `export_id` for cfg (caller-owned storage path). */
int bb_buffer_bytes(const bb_config *cfg, int32_t export_id, int64_t *bytes);

/* Create a simulator that allocates and owns all of its buffers. */
int bb_create(const bb_config *cfg, bb_sim **out);

/* Create a simulator over caller-owned buffers: bufs[id] for every id in
 * [0, BB_NUM_REFERENCE_EXPORTS) and [BB_INTERNAL_FIRST, BB_INTERNAL_LAST]
 * (nbuf = BB_INTERNAL_LAST + 1, unused slots NULL), each at least
 * bb_buffer_bytes() long, 16-byte aligned, on the simulator's device (host
 * memory in CPU mode).  Worlds are generated into them (src/gen.cpp:13-214). */
int bb_create_with_buffers(const bb_config *cfg, void *const *bufs, int32_t nbuf, bb_sim **out);

int bb_destroy(bb_sim *sim);

/* One step of every world (the task graph of src/game.cpp:1463-1526),
 * asynchronous on `stream` in CUDA mode, synchronous in CPU mode. */
int bb_step(bb_sim *sim, void *stream);

/* n steps.  If random_actions != 0, each step first overwrites the action
 * tensor with the synthetic workload threefry2x32(key={action_seed, step0+s},
 * ctr={global world, agent}) (buckets [2,8,3,2,2,2], scripts/env.py:102).
 * If kernel_ms is non-NULL (CUDA mode), HIP events bracket every step kernel
 * and the summed kernel time is written there after a stream sync. */
int bb_step_n(bb_sim *sim, int32_t n, int32_t random_actions, uint32_t action_seed,
              uint32_t step0, void *stream, float *kernel_ms);

/* Only the synthetic action write (the bench's stand-in for the Python
 * `actions[:] = ...` write of scripts/env.py:147). */
int bb_write_random_actions(bb_sim *sim, uint32_t action_seed, uint32_t step, void *stream);

/* n steps whose actions are already resident: step k reads its actions from
 * (and the defence AI writes its overrides back to) the int32 rows
 * actions + k * num_worlds * num_agents * 6 (layout [n][W][N][6], memory of the
 * simulator's device in CUDA mode, host memory in CPU mode) instead of the
 * action tensor; afterwards the action tensor holds step n-1's rows.
 * On gfx950 the n steps run as one launch, every step's outputs (each state
 * column, observation row, reward, done and action write-back) written as by
 * bb_step; identical results to n bb_step launches.  At 2 agents, and at
 * more while a step's bytes stay in the Infinity Cache, the worlds stay on
 * the chip between steps (registers: k_rollout_split / k_rollout; LDS from 4
 * agents: k_rollout_shared; BB_STAGED_RESIDENT); otherwise each wave steps its
 * worlds n times reloading the state its lanes stored (k_step_loop:
 * BB_STAGED_LOOP).  MADRONA_BB_STEP_LOOP = 0 / 1 / 2 forces one launch per
 * step / the reloading loop / the resident loop where it exists.
 * kernel_ms as in bb_step_n (the launch's). */
int bb_step_n_staged(bb_sim *sim, int32_t n, int32_t *actions, void *stream, float *kernel_ms);

/* The launch bb_step_n_staged makes for n steps on this simulator, and the
 * algorithmic bytes of that call over all worlds: n B(N) per world, less the
 * state reads of steps 1..n-1 on the resident path. */
#define BB_STAGED_PER_STEP 0 /* one step launch per step (also: CPU mode, n < 2) */
#define BB_STAGED_LOOP 1     /* one k_step_loop launch */
#define BB_STAGED_RESIDENT 2 /* one k_rollout_split / k_rollout launch, state columns stored every step */
int32_t bb_step_staged_path(const bb_sim *sim, int32_t n);
int64_t bb_step_staged_bytes(const bb_sim *sim, int32_t n);

/* Stage n steps of the synthetic workload of bb_step_n (steps step0..step0+n-1)
 * into actions[n][W][N][6] for bb_step_n_staged. */
int bb_fill_random_actions(bb_sim *sim, int32_t *actions, int32_t n, uint32_t action_seed, uint32_t step0,
                           void *stream);

/* bb_rollout flags */
#define BB_ROLLOUT_PER_STEP 0x1u /* one step kernel launch per step, state through HBM
                                    (default on gfx950 at 2 agents: one launch for all
                                    steps, the worlds held in registers) */

/* n-step rollout.  Equivalent to, for k = 0..n-1:
 *     action tensor := actions[k]; bb_step();
 *     obs_out[k] := observations; reward_out[k] := reward; done_out[k] := done
 * with the defence AI's overrides written back into actions[k] (as
 * bb_step_n_staged).  Layouts: actions int32 [n][W][N][6], obs_out float
 * [n][W][N][obs_width], reward_out/done_out float [n][W][N], on the
 * simulator's device (host memory in CPU mode).  Observation columns from
 * roundup4(61 + 38(N-1) + 2N) on are never written: zero obs_out once.  A
 * NULL output is not recorded (that tensor of the simulator is rewritten
 * every step instead).  Afterwards every simulator column holds the state
 * after step n-1 (observations, reward, done and action included).
 * kernel_ms as in bb_step_n (summed over the launches). */
int bb_rollout(bb_sim *sim, int32_t n, int32_t *actions, float *obs_out, float *reward_out, float *done_out,
               uint32_t flags, void *stream, float *kernel_ms);

/* Trajectory recorder.  One record of one world is bb_record_words(N) int32
 * words (18 N + 27): the columns scripts/ppo.py:94-105 logs, in its key order
 * and each in its export layout -- agent_pos f32[N][3], ball_pos f32[3],
 * ball_vel f32[3], orientation f32[N][4], ball_physics i32[7],
 * agent_possession i32[N][3], game_state f32[14], reward f32[N],
 * action i32[N][6], done f32[N].  bb_record copies worlds [world0,
 * world0 + count) to dst + slot * count * words (records world-major), on
 * `stream` after whatever precedes it there; host memory in CPU mode. */
int32_t bb_record_words(int32_t num_agents);
int bb_record(bb_sim *sim, int64_t world0, int32_t count, int32_t *dst, int64_t slot, void *stream);

/* Policy inference (scripts/agent.py:108-154 at num_channels = 32,
 * num_layers = 2, input 128, buckets [2,8,3,2,2,2]).  fp32 row-major
 * [out][in] weights on the device (host memory for BB_EXEC_CPU); obs_inv =
 * rsqrt(running var + 1e-5) as agent.py:30-35 computes it; head_w / head_b =
 * the 19 actor rows, the critic row, then 12 zero rows (32 x 32, 32). */
typedef struct bb_policy_weights {
    const float *obs_mean, *obs_inv;
    const float *w1, *b1, *ln1_w, *ln1_b;
    const float *w2, *b2, *ln2_w, *ln2_b;
    const float *head_w, *head_b;
} bb_policy_weights;

/* For rows r in [0, rows): reads obs + r * obs_stride (128 floats, 16-byte
 * aligned), writes 6 int32 actions to actions + r * action_stride (e.g. the
 * action tensor's column of one agent), and optionally log_prob[r] (sum over
 * the buckets) and value[r].  stochastic = 0: per-bucket argmax (best(),
 * scripts/action.py:21-23); 1: a categorical sample (Categorical.sample,
 * action.py:29-33) by inverse CDF, bucket b's uniform from threefry({seed,
 * step}, {r, b >> 1}) word b & 1.  gpu_id: the device of the pointers (CUDA
 * mode). */
int bb_policy_forward(const bb_policy_weights *w, int32_t exec_mode, int32_t gpu_id, const float *obs,
                      int64_t rows, int64_t obs_stride, int32_t *actions, int64_t action_stride, float *log_prob,
                      float *value, int32_t stochastic, uint32_t seed, uint32_t step, void *stream);

/* PPO's rollout on the device (scripts/ppo.py:61-141 over scripts/env.py:126-170;
 * the reference's 2-agent game).  For k = 0..n-1:
 *     actions, log_probs, values = agent(obs)          (policy w, trainee rows)
 *     [opponent: the frozen policy acts for the other agent, env.py:127-143]
 *     actions[:, trainee] = actions; bb_step()          (env.py:147,155)
 *     buffer.obs/actions/log_probs/values[k] = obs, actions, log_probs, values
 *     buffer.rewards/dones[k] = the trainee's reward / done after the step
 * and then next_value = agent.evaluate(obs after the last step) (ppo.py:136-137).
 * Each output is optional (NULL: not recorded; reward and done together).
 * Layouts (the simulator's device, host memory in CPU mode): obs float [n][W][128],
 * actions int32 [n][W][6] (the policy's, before the defence AI's overrides),
 * log_prob / value / reward / done float [n][W], next_value float [W].
 * Sampling as bb_policy_forward with step = step0 + k (stochastic = 0: argmax);
 * the opponent samples with seed ^ 0x9E3779B9.  Equal, bit for bit, to n x
 * (bb_policy_forward on the trainee rows; bb_step) with the reads above.
 * On gfx950 without an opponent, up to 16 384 worlds one fused launch runs
 * all n steps with the worlds in registers (BB_PPO_PATH_FUSED_ROLLOUT); above,
 * a policy launch and then one launch in which every wave runs its worlds' n
 * steps, each followed by the next policy pass on the rows in LDS
 * (BB_PPO_PATH_FUSED_STEP).  flags BB_ROLLOUT_PER_STEP forces a policy launch
 * and a step launch per step instead (so does an opponent); from 32 768
 * worlds those per-step launches of two world halves go to `stream` and to a
 * second stream the simulator owns (created on first use, destroyed by
 * bb_destroy); `stream` waits for both before the call's last work, so stream
 * order holds for the caller.
 * kernel_ms (CUDA mode): time from the first launch to the last, after a sync. */
typedef struct bb_policy_rollout_buffers {
    float *obs;
    int32_t *actions;
    float *log_prob, *value, *reward, *done, *next_value;
} bb_policy_rollout_buffers;
int bb_rollout_policy(bb_sim *sim, const bb_policy_weights *w, const bb_policy_weights *opponent, int32_t n,
                      int32_t trainee, int32_t stochastic, uint32_t seed, uint32_t step0,
                      const bb_policy_rollout_buffers *out, uint32_t flags, void *stream, float *kernel_ms);

/* The implementation bb_rollout_policy takes on this simulator, and the
 * algorithmic bytes of one call of n steps with every output recorded (the
 * bytes that path must move: HBM roofline of the PPO loop).
 * On a simulator of other than 2 agents both fail: BB_ERR_UNSUPPORTED (< 0),
 * bb_last_error() says why. */
#define BB_PPO_PATH_HOST 0          /* CPU mode: the host executor */
#define BB_PPO_PATH_FUSED_ROLLOUT 1 /* one k_rollout_policy launch for all n steps */
#define BB_PPO_PATH_FUSED_STEP 2    /* a policy launch, then k_rollout_ppo (step + next policy pass, n times) */
#define BB_PPO_PATH_PER_STEP 3      /* a policy launch and a step launch per step */
int32_t bb_rollout_policy_path(const bb_sim *sim, int32_t with_opponent, uint32_t flags);
int64_t bb_rollout_policy_bytes(const bb_sim *sim, int32_t with_opponent, uint32_t flags, int32_t n);

int bb_set_action(bb_sim *sim, int32_t world_idx, int32_t agent_idx, int32_t move_speed,
                  int32_t move_angle, int32_t rotate, int32_t grab, int32_t pass,
                  int32_t shoot, void *stream);

int bb_trigger_reset(bb_sim *sim, int32_t world_idx, void *stream);

/* Describe one export: data pointer (aliasing the live state), dtype and
 * reference shape (src/mgr.cpp:317-445; ndim <= 3, dims[ndim..3] = 0). */
int bb_export(bb_sim *sim, int32_t export_id, void **ptr, int32_t *dtype, int32_t *ndim,
              int64_t dims[4]);

/* Accessors. */
int64_t bb_num_worlds(const bb_sim *sim);
int32_t bb_num_agents(const bb_sim *sim);
int32_t bb_exec_mode(const bb_sim *sim);

/* Algorithmic HBM bytes moved by one step of one world (roofline). */
int64_t bb_algorithmic_bytes_per_world(int32_t num_agents);

/* 1 if bb_rollout runs as one fused launch (gfx950) for num_agents. */
int32_t bb_rollout_fused(int32_t num_agents);

/* Algorithmic HBM bytes of a fused rollout (roofline): per world
 * and step (action row in, observation row + reward + done out), and per
 * world and launch (the remaining state columns, in once and out once). */
int64_t bb_rollout_bytes_per_world_step(int32_t num_agents);
int64_t bb_rollout_state_bytes_per_world(int32_t num_agents);

/* Message for the last error on this thread ("" if none). */
const char *bb_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
