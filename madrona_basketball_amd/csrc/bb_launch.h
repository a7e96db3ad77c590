// bb_launch.h -- host-side entry points into the gfx950 kernels
// (bb_kernels.hip, one translation unit per agent count) and the host executor.
#pragma once
#include <hip/hip_runtime.h>
#include "bb_sim.h"
#include "bb_policy.h"

namespace bb {

// Kernel variants of k_step (diagnostics for the roofline analysis; MODE_FULL
// is the product kernel).
enum StepMode : int {
    MODE_FULL = 0,        // 19 systems, observation rows staged through LDS
    MODE_IO = 1,          // load + store of every column only
    MODE_IO_OBS = 2,      // load + observation rows + store, no systems
    MODE_DIRECT_OBS = 3,  // 19 systems, observation rows stored lane-strided (v1)
    MODE_NO_OBS = 4,      // systems 1-17 and 19, no observation rows
    MODE_SKIP = 5,        // full, minus the systems whose bit is set in Params::diag_skip
    MODE_TRACE = 6,       // full, plus per-wave phase clocks into Params::diag_ts
};

// K-step rollout (bb_rollout): step t reads actions + t*W*N*6 and writes its
// observation rows, rewards and done flags at obs/reward/done + t*(row stride).
// The N = 2 K-step rollout kernels store the last step's rows into the sim's
// observation tensor as well as the recorded buffer (instead of a copy after
// the launch: 65 536 x 2 worlds 18.1 -> 17.3 us per step, 8 192 x 2 6.2 -> 5.55).
struct RolloutArgs {
    int32_t *actions;  // [K][W][N][6]   (defence overrides written back)
    float *obs;        // [K][W][N][OBSW]
    float *reward;     // [K][W][N]
    float *done;       // [K][W][N]
    int64_t obs_step;  // floats between consecutive steps' obs (0: one buffer for all steps)
    int64_t rd_step;   // floats between consecutive steps' reward/done (0: likewise)
    int32_t steps;     // K
    // bb_step_n_staged's register-resident loop: every step also stores the
    // state columns, so each step leaves in memory exactly what a k_step launch
    // would (the state itself stays in registers between steps).  Then reward
    // and done must be the sim's own columns (rd_step 0): they are stored with
    // the state; the action rows are stored whole into actions[t], as k_step.
    int32_t store_state;
};

// PPO rollout with the policy in the loop (bb_rollout_policy, fused kernel
// k_rollout_policy<2>): per step the policy on the trainee rows, the step, the
// buffer stores of scripts/ppo.py:129-134; then next_value.
struct PolicyRolloutArgs {
    PolicyWeights w;
    float *obs_out;       // [K][W][128]  trainee observation before each step
    int32_t *act_out;     // [K][W][6]    the policy's actions
    float *log_prob, *value, *reward, *done;  // [K][W]
    float *next_value;    // [W]
    int32_t steps, trainee, stochastic;
    uint32_t seed, step0;
};

// One step of PPO's rollout loop with the policy fused behind it
// (k_step_ppo<2> / k_rollout_ppo<2>, bb_rollout_policy above 16 384 worlds): step k on the
// trainee's actions already in the sim's action column, then the policy on the
// trainee's rows after the step (scripts/ppo.py:65-134 over env.py:126-170) --
// the actions of step k + 1 into the action column, buffer.obs/actions/
// log_probs/values[k + 1] -- or, after the rollout's last step, the value only
// (next_value, ppo.py:136-137).  All output pointers optional.
struct PpoStepArgs {
    PolicyWeights w;
    float *reward, *done;       // [W] buffer.rewards / not_dones source of step k (the trainee's)
    float *obs_rec;             // [W][128] buffer.obs[k + 1] (not on the last step)
    int32_t *act_out;           // [W][6]   buffer.actions[k + 1]
    float *log_prob, *value;    // [W]      buffer.log_probs / values[k + 1], or next_value on the last step
    int32_t trainee, stochastic;
    int32_t last;               // the rollout's last step: every row into the sim's obs, value only
    uint32_t seed, step;        // the policy's sampling key (seed, step0 + k + 1)
    float *value_last;          // k_rollout_ppo: next_value (the value output of its last step)
    // k_rollout_ppo: the policy pass of step 0 in the launch (on the sim's rows
    // of the trainee before the first step, key step0): buffer.obs / actions /
    // log_probs / values[0] (each optional); pass0 = 0: done by a launch before
    int32_t pass0;
    uint32_t step0;
    float *obs0;
    int32_t *act0;
    float *log_prob0, *value0;
};
// N = 2 only (hipErrorNotSupported otherwise)
hipError_t launch_step_ppo(int n, const Params &p, const PpoStepArgs &a, hipStream_t s);
// The `steps` steps of a rollout in one launch (k_rollout_ppo<2>): `a` holds
// step 0's arguments (outputs of step k at k x W past them; its `last` is
// ignored), value_last the next_value output.  N = 2 only.
hipError_t launch_rollout_ppo(int n, const Params &p, const PpoStepArgs &a, int32_t steps, hipStream_t s);

// Trajectory recorder (bb_record): NSEG column segments per recorded world.
constexpr int RECORD_SEGS = 10;
struct RecordArgs {
    const uint32_t *src[RECORD_SEGS];  // column bases
    int32_t wpw[RECORD_SEGS];          // words per world of each column
    int32_t off[RECORD_SEGS + 1];      // word offset of each segment in a record
};
int32_t record_words(int n);
RecordArgs record_args(const Params &p, int n);

// Path overrides, for tests and A/B timing only: set through the C ABI's
// bb_diag_set (not in the public header), never read from the environment.
// -1 (the initial value) = the product's own rule for that choice.
enum DiagKey : int {
    DIAG_STEP_LOOP = 0,                  // bb_step_n_staged's launch: BB_STAGED_* (0 per step, 1 k_step_loop, 2 resident)
    DIAG_ROLLOUT_SPLIT = 1,              // k_rollout_split: 0 never, 1 always (else while its grid fits 2 per CU)
    DIAG_ROLLOUT_MINW = 2,               // k_rollout's register budget: 1 or 2 waves per SIMD
    DIAG_ROLLOUT_SHARED_MAX_N = 3,       // the N >= 4 K-step rollout kernel up to this many agents (default 4)
    DIAG_PPO_PWAVES = 4,                 // k_rollout_policy's policy waves: 2 or 4
    DIAG_PPO_FUSED_MAX_WORLDS = 5,       // k_rollout_policy up to this many worlds (default 16 384)
    DIAG_PPO_STEP_FUSED_MIN_WORLDS = 6,  // the fused PPO step from this many worlds (default 1; 0 never)
    DIAG_PPO_STEP_LOOP = 7,              // 0: one k_step_ppo launch per step instead of one k_rollout_ppo
    DIAG_POLICY_WG = 8,                  // k_policy_wg: 0 never, 1 always (else from 98 304 rows)
    DIAG_KEYS = 9
};
extern int diag_override[DIAG_KEYS];
inline int diag_or(int key, int dflt)
{
    const int v = diag_override[key];
    return v >= 0 ? v : dflt;
}

template <int N> hipError_t launch_step_t(const Params &p, int mode, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1);
template <int N> hipError_t launch_init_t(const Params &p, hipStream_t s);
// `steps` staged steps (actions + t * W * N * 6) in one launch (k_step_loop;
// N = 2 only, hipErrorNotSupported otherwise)
template <int N> hipError_t launch_step_loop_t(const Params &p, int32_t *actions, int32_t steps, hipStream_t s,
                                               hipEvent_t ev0, hipEvent_t ev1);
template <int N> int step_grid(int64_t num_worlds);  // k_step workgroups (= waves)
template <int N> hipError_t launch_rollout_t(const Params &p, const RolloutArgs &r, hipStream_t s, hipEvent_t ev0,
                                             hipEvent_t ev1);
template <int N> bool fused_rollout();  // k_rollout<N> exists (else: one k_step launch per step)
// The K-step rollout kernel family a grid takes (launch_rollout_t; its
// RolloutArgs::store_state instances for the resident loop).
enum RolloutKernel : int {
    RK_NONE = -1,   // no fused rollout: one k_step launch per step
    RK_SPLIT = 0,   // k_rollout_split<N> (sim wave + row wave per 32 worlds)
    RK_MINW1 = 1,   // k_rollout<N, 1>: the whole register file, at most one wave per SIMD
    RK_MINW2 = 2,   // k_rollout<N, 2>
    RK_SHARED = 3,  // k_rollout_shared<N> (N >= 4, the world in LDS)
};
template <int N> int rollout_kernel_t(int64_t num_worlds);
// bb_step_n_staged's register-resident loop (RolloutArgs::store_state) is taken
template <int N> bool resident_staged(int64_t num_worlds);
template <int N> bool step_records_t();  // k_step<N> honours Params::rec_obs
template <int N> hipError_t launch_rollout_policy_t(const Params &p, const PolicyRolloutArgs &r, hipStream_t s);

#define BB_EXTERN_N(n)                                                                  \
    extern template hipError_t launch_step_t<n>(const Params &, int, hipStream_t, hipEvent_t, hipEvent_t); \
    extern template hipError_t launch_init_t<n>(const Params &, hipStream_t);           \
    extern template hipError_t launch_step_loop_t<n>(const Params &, int32_t *, int32_t, hipStream_t, hipEvent_t, hipEvent_t); \
    template <> int step_grid<n>(int64_t);                                              \
    extern template hipError_t launch_rollout_t<n>(const Params &, const RolloutArgs &, hipStream_t, hipEvent_t, hipEvent_t); \
    extern template int rollout_kernel_t<n>(int64_t);                                   \
    template <> bool fused_rollout<n>();                                                \
    template <> bool resident_staged<n>(int64_t);                                       \
    template <> bool step_records_t<n>();                                               \
    extern template hipError_t launch_rollout_policy_t<n>(const Params &, const PolicyRolloutArgs &, hipStream_t);
BB_EXTERN_N(2)
BB_EXTERN_N(4)
BB_EXTERN_N(6)
BB_EXTERN_N(8)
BB_EXTERN_N(10)
#undef BB_EXTERN_N

hipError_t launch_step(int n, const Params &p, hipStream_t s, int mode = MODE_FULL, hipEvent_t ev0 = nullptr,
                       hipEvent_t ev1 = nullptr);
hipError_t launch_init(int n, const Params &p, hipStream_t s);
hipError_t launch_step_loop(int n, const Params &p, int32_t *actions, int32_t steps, hipStream_t s,
                            hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
hipError_t launch_rollout(int n, const Params &p, const RolloutArgs &r, hipStream_t s, hipEvent_t ev0 = nullptr,
                          hipEvent_t ev1 = nullptr);
bool fused_rollout_n(int n);
int rollout_kernel_n(int n, int64_t num_worlds);
bool resident_staged_n(int n, int64_t num_worlds);
// whether k_step honours Params::rec_obs (PPO's buffer.obs record from the
// step's row passes): the agent-lane kernel of the 2-agent game only
bool step_records(int n);
// fused PPO rollout (N = 2 only; hipErrorNotSupported otherwise)
hipError_t launch_rollout_policy(int n, const Params &p, const PolicyRolloutArgs &r, hipStream_t s);
int step_grid_n(int n, int64_t num_worlds);
hipError_t launch_random_actions(int n, const Params &p, uint32_t seed, uint32_t step, hipStream_t s);
hipError_t launch_poke(int32_t *dst, int count, const int32_t *vals, hipStream_t s);
hipError_t launch_policy(const PolicyArgs &a, hipStream_t s);
void host_policy(const PolicyArgs &a);
hipError_t launch_record(const RecordArgs &a, int64_t world0, int32_t count, uint32_t *dst, hipStream_t s);
void host_record(const RecordArgs &a, int64_t world0, int32_t count, uint32_t *dst);
// diagnostics: the step's scalar math on the device (bb_diag_math)
hipError_t launch_math_probe(int fn, const float *x, const float *y, float *out, int64_t n, hipStream_t s);
// diagnostics: bbm's short-path divide / square root vs IEEE (bb_diag_divsqrt)
hipError_t launch_divsqrt_probe(int mode, uint64_t start, uint64_t count, uint32_t seed, uint32_t *counts,
                                uint32_t *ex, int blocks, hipStream_t s);
// streaming copy with the step's traffic mix (read_b, write_b bytes per item)
hipError_t launch_stream_probe(const float4 *src, float4 *dst, int64_t items, int read_q, int write_q, int pattern,
                               int nt, hipStream_t s);

// Host executor (ExecMode.CPU): the same step code over a persistent thread
// pool (bb_host.hip HostPool); with `actions` each worker first writes the
// synthetic action rows of its own worlds.
class HostPool;
int host_step(int n, const Params &p, HostPool &pool, bool actions = false, uint32_t seed = 0, uint32_t step = 0);
int host_steps(int n, const Params &p, HostPool &pool, int32_t steps, bool actions, uint32_t seed, uint32_t step0);
int host_init(int n, const Params &p);
int host_random_actions(int n, const Params &p, HostPool &pool, uint32_t seed, uint32_t step);

}  // namespace bb
