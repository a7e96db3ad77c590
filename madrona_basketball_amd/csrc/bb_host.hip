// bb_host.hip -- C ABI (include/madrona_basketball_amd.h) and the host executor.
//
// The ABI replaces the reference's Manager + nanobind class
// (src/mgr.cpp:236-445, src/bindings.cpp:17-101).  Buffers are either owned
// (bb_create: hipMalloc / aligned host memory) or borrowed from the caller
// (bb_create_with_buffers: the Python layer hands in torch allocations so
// that `to_torch()` views are native torch tensors).  In CUDA mode every
// operation is enqueued on the caller's stream; nothing here synchronises
// except creation and the optional kernel timing of bb_step_n.
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/madrona_basketball_amd.h"
#include "bb_launch.h"
#include "bb_sim.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char *what)
{
    return fail(BB_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

constexpr int NUM_SLOTS = BB_INTERNAL_LAST + 1;

bool slot_used(int id)
{
    return (id >= 0 && id < BB_NUM_REFERENCE_EXPORTS) || (id >= BB_INTERNAL_FIRST && id <= BB_INTERNAL_LAST);
}

// Reference tensor shapes (src/mgr.cpp:317-445) + internal columns.
bool export_info(int id, int n, int64_t W, int32_t *dtype, int32_t *ndim, int64_t dims[4], int64_t *words_per_world)
{
    const int64_t ow = bb::obs_width(n);
    int32_t dt = BB_DTYPE_INT32, nd = 3;
    int64_t d1 = n, d2 = 0;
    switch (id) {
    case BB_EXPORT_RESET: d2 = 1; break;
    case BB_EXPORT_GAME_STATE: dt = BB_DTYPE_FLOAT32; nd = 2; d1 = 14; break;
    case BB_EXPORT_ACTION: d2 = 6; break;
    case BB_EXPORT_ACTION_MASK: d2 = 4; break;
    case BB_EXPORT_AGENT_POS: dt = BB_DTYPE_FLOAT32; d2 = 3; break;
    case BB_EXPORT_OBSERVATIONS: dt = BB_DTYPE_FLOAT32; d2 = ow; break;
    case BB_EXPORT_REWARD: dt = BB_DTYPE_FLOAT32; nd = 2; break;
    case BB_EXPORT_DONE: dt = BB_DTYPE_FLOAT32; nd = 2; break;
    case BB_EXPORT_AGENT_ENTITY_ID: nd = 2; break;
    case BB_EXPORT_AGENT_POSSESSION: d2 = 3; break;
    case BB_EXPORT_ORIENTATION: dt = BB_DTYPE_FLOAT32; d2 = 4; break;
    case BB_EXPORT_TEAM: d2 = 5; break;
    case BB_EXPORT_AGENT_STATS: d2 = 2; break;
    case BB_EXPORT_BALL_POS: dt = BB_DTYPE_FLOAT32; d1 = 1; d2 = 3; break;
    case BB_EXPORT_BALL_PHYSICS: d1 = 1; d2 = 7; break;
    case BB_EXPORT_BALL_ENTITY_ID: nd = 2; d1 = 1; break;
    case BB_EXPORT_BALL_GRABBED: d1 = 1; d2 = 2; break;
    case BB_EXPORT_BALL_VELOCITY: dt = BB_DTYPE_FLOAT32; d1 = 1; d2 = 3; break;
    case BB_EXPORT_HOOP_POS: dt = BB_DTYPE_FLOAT32; d1 = 2; d2 = 3; break;
    case BB_INTERNAL_AGENT_VELOCITY: dt = BB_DTYPE_FLOAT32; d2 = 3; break;
    case BB_INTERNAL_GRAB_COOLDOWN: dt = BB_DTYPE_FLOAT32; nd = 2; break;
    case BB_INTERNAL_CUR_STEP: nd = 2; break;
    case BB_INTERNAL_INBOUNDING: d2 = 2; break;
    case BB_INTERNAL_ATTRIBUTES: dt = BB_DTYPE_FLOAT32; d2 = 10; break;
    case BB_INTERNAL_WORLD_CLOCK: nd = 1; d1 = 0; break;
    case BB_INTERNAL_RNG_COUNTER: nd = 1; d1 = 0; break;
    default: return false;
    }
    if (dtype) *dtype = dt;
    if (ndim) *ndim = nd;
    if (dims) {
        dims[0] = W; dims[1] = nd >= 2 ? d1 : 0; dims[2] = nd >= 3 ? d2 : 0; dims[3] = 0;
    }
    if (words_per_world) *words_per_world = (nd == 1) ? 1 : (nd == 2 ? d1 : d1 * d2);
    return true;
}

bool valid_agents(int n) { return n == 2 || n == 4 || n == 6 || n == 8 || n == 10; }

int validate(const bb_config *cfg)
{
    if (!cfg) return fail(BB_ERR_INVALID_ARG, "config is NULL");
    if (cfg->num_worlds < 1) return fail(BB_ERR_INVALID_ARG, "num_worlds must be >= 1");
    if (cfg->discrete_x < 1 || cfg->discrete_y < 1) return fail(BB_ERR_INVALID_ARG, "discrete_x/discrete_y must be >= 1");
    if (!valid_agents(cfg->num_agents))
        return fail(BB_ERR_UNSUPPORTED, "num_agents must be one of 2, 4, 6, 8, 10 (reference: 2)");
    if (cfg->exec_mode != BB_EXEC_CPU && cfg->exec_mode != BB_EXEC_CUDA)
        return fail(BB_ERR_INVALID_ARG, "exec_mode must be BB_EXEC_CPU or BB_EXEC_CUDA");
    if (cfg->flags & ~(BB_FLAG_PER_WORLD_RNG | BB_FLAG_NO_TAG_MASK | BB_FLAG_FULL_GAME))
        return fail(BB_ERR_INVALID_ARG, "unknown flag bits");
    return BB_OK;
}

int host_threads_for(int64_t worlds)
{
    // default: the machine's threads, at most 16 (a GPU box's CPU share);
    // BB_CPU_THREADS overrides
    const char *env = std::getenv("BB_CPU_THREADS");
    int t = env ? std::atoi(env) : (int)std::thread::hardware_concurrency();
    if (!env && t > 16) t = 16;
    if (t < 1) t = 1;
    const int64_t max_useful = (worlds + 255) / 256;
    if (t > max_useful) t = (int)max_useful;
    return t < 1 ? 1 : t;
}

struct DeviceGuard {
    int prev = -1;
    bool active = false;
    explicit DeviceGuard(int dev)
    {
        if (dev < 0) return;
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) {
            if (hipSetDevice(dev) == hipSuccess) active = true;
        }
    }
    ~DeviceGuard()
    {
        if (active) (void)hipSetDevice(prev);
    }
};

}  // namespace

namespace bb {

// Persistent worker pool of the host executor (ExecMode.CPU), the stand-in
// for the reference's CPU TaskGraphExecutor worker threads (src/mgr.cpp:49-81:
// created once with the Manager, reused every step).  run(f) calls f(t) for
// t = 0..size-1 on the workers -- the calling thread is worker 0 -- and
// returns when all are done.  Workers spin briefly, then sleep on a condition
// variable, between jobs.
class HostPool {
public:
    explicit HostPool(int n) : n_(n < 1 ? 1 : n)
    {
        // (threads pinned to CPUs measured slower on the GPU box's 16-core
        // share: 46.9 M pinned against 52-61 M env-steps/s unpinned,
        // profiles/r03/final_bench.log)
        for (int t = 1; t < n_; t++) th_.emplace_back([this, t] { worker(t); });
    }
    ~HostPool()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return n_; }
    void run(const std::function<void(int)> &f)
    {
        if (n_ == 1) { f(0); return; }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &f;
            left_.store(n_ - 1, std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        f(0);
        // the others: spin, then sleep
        for (int i = 0; left_.load(std::memory_order_acquire) != 0; i++) {
            if (i > 4096) {
                std::unique_lock<std::mutex> g(m_);
                done_cv_.wait(g, [this] { return left_.load(std::memory_order_acquire) == 0; });
                break;
            }
            std::this_thread::yield();
        }
        job_ = nullptr;
    }

private:
    void worker(int t)
    {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g = gen_.load(std::memory_order_acquire);
            for (int i = 0; g == seen && i < 4096; i++) {
                std::this_thread::yield();
                g = gen_.load(std::memory_order_acquire);
            }
            if (g == seen) {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
                g = gen_.load(std::memory_order_acquire);
            }
            seen = g;
            const std::function<void(int)> *job;
            {
                std::lock_guard<std::mutex> lk(m_);
                if (stop_) return;
                job = job_;
            }
            (*job)(t);
            if (left_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> lk(m_);
                done_cv_.notify_one();
            }
        }
    }
    const int n_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> left_{0};
    const std::function<void(int)> *job_ = nullptr;
    bool stop_ = false;
};

}  // namespace bb

struct bb_sim {
    bb_config cfg;
    int n = 2;
    int device = -1;
    bool owns = false;
    void *slot[NUM_SLOTS] = {};
    bb::Params p;
    std::unique_ptr<bb::HostPool> pool;  // ExecMode.CPU workers (created with the simulator)
    // (CUDA mode) the second stream and events of bb_rollout_policy's split
    // per-step loop, created on first use
    static constexpr int MAX_PARTS = 4;
    hipStream_t aux[MAX_PARTS - 1] = {};
    hipEvent_t aux_ev[2 * MAX_PARTS] = {};
};

namespace {

void bind_params(bb_sim *s)
{
    bb::Params &p = s->p;
    std::memset(&p, 0, sizeof(p));
    bb::Columns &c = p.c;
    void **b = s->slot;
    c.reset = (int32_t *)b[BB_EXPORT_RESET];
    c.game_state = (uint32_t *)b[BB_EXPORT_GAME_STATE];
    c.action = (int32_t *)b[BB_EXPORT_ACTION];
    c.action_mask = (int32_t *)b[BB_EXPORT_ACTION_MASK];
    c.agent_pos = (float *)b[BB_EXPORT_AGENT_POS];
    c.obs = (float *)b[BB_EXPORT_OBSERVATIONS];
    c.reward = (float *)b[BB_EXPORT_REWARD];
    c.done = (float *)b[BB_EXPORT_DONE];
    c.agent_id = (int32_t *)b[BB_EXPORT_AGENT_ENTITY_ID];
    c.possession = (int32_t *)b[BB_EXPORT_AGENT_POSSESSION];
    c.orientation = (float *)b[BB_EXPORT_ORIENTATION];
    c.team = (uint32_t *)b[BB_EXPORT_TEAM];
    c.stats = (float *)b[BB_EXPORT_AGENT_STATS];
    c.ball_pos = (float *)b[BB_EXPORT_BALL_POS];
    c.ball_physics = (int32_t *)b[BB_EXPORT_BALL_PHYSICS];
    c.ball_id = (int32_t *)b[BB_EXPORT_BALL_ENTITY_ID];
    c.ball_grabbed = (int32_t *)b[BB_EXPORT_BALL_GRABBED];
    c.ball_vel = (float *)b[BB_EXPORT_BALL_VELOCITY];
    c.hoop_pos = (float *)b[BB_EXPORT_HOOP_POS];
    c.agent_vel = (float *)b[BB_INTERNAL_AGENT_VELOCITY];
    c.cooldown = (float *)b[BB_INTERNAL_GRAB_COOLDOWN];
    c.cur_step = (uint32_t *)b[BB_INTERNAL_CUR_STEP];
    c.inbounding = (int32_t *)b[BB_INTERNAL_INBOUNDING];
    c.attributes = (float *)b[BB_INTERNAL_ATTRIBUTES];
    c.world_clock = (int32_t *)b[BB_INTERNAL_WORLD_CLOCK];
    c.rng_counter = (uint32_t *)b[BB_INTERNAL_RNG_COUNTER];
    const bb_config &cfg = s->cfg;
    p.num_worlds = cfg.num_worlds;
    p.world_offset = cfg.world_offset;
    // bindings.cpp:28-33: cellsPerMeter = 1, width/height = discrete cells
    p.width = (float)cfg.discrete_x / (float)1;
    p.height = (float)cfg.discrete_y / (float)1;
    p.start_x = cfg.start_x;
    p.start_y = cfg.start_y;
    // hoop positions (src/gen.cpp:96-141)
    const float csx = (p.width - bb::COURT_L) / 2.0f;
    const float ccy = p.height / 2.0f;
    p.hoop0[0] = csx + bb::HOOP_FROM_BASE; p.hoop0[1] = ccy; p.hoop0[2] = 0.f;
    p.hoop1[0] = csx + bb::COURT_L - bb::HOOP_FROM_BASE; p.hoop1[1] = ccy; p.hoop1[2] = 0.f;
    p.seed = cfg.rand_seed;
    p.flags = cfg.flags;
    bb::build_tables(p);
}

int64_t slot_bytes(const bb_config *cfg, int id)
{
    int64_t wpw = 0;
    if (!export_info(id, cfg->num_agents, cfg->num_worlds, nullptr, nullptr, nullptr, &wpw)) return -1;
    return wpw * 4 * cfg->num_worlds;
}

int init_worlds(bb_sim *s)
{
    if (s->cfg.exec_mode == BB_EXEC_CUDA) {
        DeviceGuard g(s->device);
        for (int id = 0; id < NUM_SLOTS; id++) {
            if (!slot_used(id)) continue;
            hipError_t e = hipMemsetAsync(s->slot[id], 0, (size_t)slot_bytes(&s->cfg, id), nullptr);
            if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync");
        }
        hipError_t e = bb::launch_init(s->n, s->p, nullptr);
        if (e != hipSuccess) return hip_fail(e, "launch init kernel");
        e = hipDeviceSynchronize();
        if (e != hipSuccess) return hip_fail(e, "world generation");
        return BB_OK;
    }
    for (int id = 0; id < NUM_SLOTS; id++)
        if (slot_used(id)) std::memset(s->slot[id], 0, (size_t)slot_bytes(&s->cfg, id));
    return bb::host_init(s->n, s->p);
}

int create_common(const bb_config *cfg, void *const *bufs, int32_t nbuf, bb_sim **out)
{
    if (!out) return fail(BB_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    int rc = validate(cfg);
    if (rc != BB_OK) return rc;
    bb_sim *s = new bb_sim();
    s->cfg = *cfg;
    s->n = cfg->num_agents;
    s->owns = bufs == nullptr;
    if (cfg->exec_mode == BB_EXEC_CUDA) {
        int count = 0;
        hipError_t e = hipGetDeviceCount(&count);
        if (e != hipSuccess || count == 0) {
            delete s;
            return fail(BB_ERR_HIP, "ExecMode.CUDA requested but no HIP device is available");
        }
        int dev = cfg->gpu_id;
        if (dev < 0) {
            if (hipGetDevice(&dev) != hipSuccess) dev = 0;
        }
        if (dev >= count) {
            delete s;
            return fail(BB_ERR_INVALID_ARG, "gpu_id out of range");
        }
        s->device = dev;
    }
    for (int id = 0; id < NUM_SLOTS; id++) {
        if (!slot_used(id)) continue;
        const int64_t bytes = slot_bytes(cfg, id);
        if (bufs) {
            if (id >= nbuf || !bufs[id]) {
                bb_destroy(s);
                return fail(BB_ERR_INVALID_ARG, "missing caller buffer for export id " + std::to_string(id));
            }
            if (((uintptr_t)bufs[id]) & 15u) {
                bb_destroy(s);
                return fail(BB_ERR_INVALID_ARG, "caller buffer for export id " + std::to_string(id) + " is not 16-byte aligned");
            }
            s->slot[id] = bufs[id];
        } else if (cfg->exec_mode == BB_EXEC_CUDA) {
            DeviceGuard g(s->device);
            void *ptr = nullptr;
            hipError_t e = hipMalloc(&ptr, (size_t)bytes);
            if (e != hipSuccess) {
                bb_destroy(s);
                return fail(BB_ERR_OOM, std::string("hipMalloc failed: ") + hipGetErrorString(e));
            }
            s->slot[id] = ptr;
        } else {
            void *ptr = std::aligned_alloc(64, (size_t)((bytes + 63) & ~int64_t(63)));
            if (!ptr) {
                bb_destroy(s);
                return fail(BB_ERR_OOM, "host allocation failed");
            }
            s->slot[id] = ptr;
        }
    }
    bind_params(s);
    if (cfg->exec_mode == BB_EXEC_CPU) s->pool.reset(new bb::HostPool(host_threads_for(cfg->num_worlds)));
    rc = init_worlds(s);
    if (rc != BB_OK) {
        bb_destroy(s);
        return rc;
    }
    *out = s;
    return BB_OK;
}

}  // namespace

// ---------------------------------------------------------------- host executor
namespace bb {

template <int N>
static void host_range(const Params &p, int64_t lo, int64_t hi)
{
    for (int64_t w = lo; w < hi; w++) step_one_world<N>(p, w);
}

// One step of every world on the pool: worker t steps worlds [W t/T, W (t+1)/T).
// With `actions` (random_actions != 0) each worker first writes its own worlds'
// synthetic action rows -- worlds are independent, so no barrier between the
// two.
template <int N>
static int host_step_n(const Params &p, HostPool &pool, bool actions, uint32_t seed, uint32_t step)
{
    const int64_t W = p.num_worlds;
    const int T = pool.size();
    pool.run([&](int t) {
        const int64_t lo = W * t / T, hi = W * (t + 1) / T;
        if (actions)
            for (int64_t w = lo; w < hi; w++)
                for (int a = 0; a < N; a++)
                    random_action(seed, step, (uint32_t)(p.world_offset + w), (uint32_t)a, p.c.action + (w * N + a) * 6);
        host_range<N>(p, lo, hi);
    });
    return BB_OK;
}

template <int N>
static int host_init_n(const Params &p)
{
    for (int64_t w = 0; w < p.num_worlds; w++) init_world<N>(p, w);
    return BB_OK;
}

// `steps` consecutive steps, each world stepped `steps` times in a row by
// its worker (optionally writing its synthetic action rows before each):
// worlds share nothing, so this equals `steps` passes over all worlds, with a
// world's state staying in the core's caches between its steps instead of
// every step streaming the thread's whole range (measured below).
template <int N>
static int host_steps_blocked(const Params &p, HostPool &pool, int32_t steps, bool actions, uint32_t seed,
                              uint32_t step0)
{
    const int64_t W = p.num_worlds;
    const int T = pool.size();
    pool.run([&](int t) {
        const int64_t lo = W * t / T, hi = W * (t + 1) / T;
        for (int64_t w = lo; w < hi; w++) {
            for (int32_t k = 0; k < steps; k++) {
                if (actions)
                    for (int a = 0; a < N; a++)
                        random_action(seed, step0 + (uint32_t)k, (uint32_t)(p.world_offset + w), (uint32_t)a,
                                      p.c.action + (w * N + a) * 6);
                step_one_world<N>(p, w);
            }
        }
    });
    return BB_OK;
}

int host_steps(int n, const Params &p, HostPool &pool, int32_t steps, bool actions, uint32_t seed, uint32_t step0)
{
    switch (n) {
    case 2: return host_steps_blocked<2>(p, pool, steps, actions, seed, step0);
    case 4: return host_steps_blocked<4>(p, pool, steps, actions, seed, step0);
    case 6: return host_steps_blocked<6>(p, pool, steps, actions, seed, step0);
    case 8: return host_steps_blocked<8>(p, pool, steps, actions, seed, step0);
    case 10: return host_steps_blocked<10>(p, pool, steps, actions, seed, step0);
    default: return BB_ERR_UNSUPPORTED;
    }
}

int host_step(int n, const Params &p, HostPool &pool, bool actions, uint32_t seed, uint32_t step)
{
    switch (n) {
    case 2: return host_step_n<2>(p, pool, actions, seed, step);
    case 4: return host_step_n<4>(p, pool, actions, seed, step);
    case 6: return host_step_n<6>(p, pool, actions, seed, step);
    case 8: return host_step_n<8>(p, pool, actions, seed, step);
    case 10: return host_step_n<10>(p, pool, actions, seed, step);
    default: return BB_ERR_UNSUPPORTED;
    }
}

int host_init(int n, const Params &p)
{
    switch (n) {
    case 2: return host_init_n<2>(p);
    case 4: return host_init_n<4>(p);
    case 6: return host_init_n<6>(p);
    case 8: return host_init_n<8>(p);
    case 10: return host_init_n<10>(p);
    default: return BB_ERR_UNSUPPORTED;
    }
}

int host_random_actions(int n, const Params &p, HostPool &pool, uint32_t seed, uint32_t step)
{
    const int64_t W = p.num_worlds;
    const int T = pool.size();
    pool.run([&](int t) {
        for (int64_t w = W * t / T; w < W * (t + 1) / T; w++)
            for (int a = 0; a < n; a++)
                random_action(seed, step, (uint32_t)(p.world_offset + w), (uint32_t)a, p.c.action + (w * n + a) * 6);
    });
    return BB_OK;
}

}  // namespace bb

// ---------------------------------------------------------------- C ABI
extern "C" {

int bb_default_config(bb_config *cfg)
{
    if (!cfg) return fail(BB_ERR_INVALID_ARG, "config is NULL");
    std::memset(cfg, 0, sizeof(*cfg));
    // scripts/env.py:20-35 with src/constants.py WORLD_WIDTH_M/HEIGHT_M
    cfg->discrete_x = 32;
    cfg->discrete_y = 17;
    cfg->start_x = (float)(31.515 / 2.0);
    cfg->start_y = (float)(16.764000000000003 / 2.0);
    cfg->max_episode_length = 39600;
    cfg->exec_mode = BB_EXEC_CPU;
    cfg->gpu_id = 0;
    cfg->num_worlds = 1;
    cfg->world_offset = 0;
    cfg->rand_seed = 0;
    cfg->flags = 0;
    cfg->num_agents = 2;
    return BB_OK;
}

int32_t bb_obs_width(int32_t num_agents) { return bb::obs_width(num_agents); }

int bb_buffer_bytes(const bb_config *cfg, int32_t export_id, int64_t *bytes)
{
    int rc = validate(cfg);
    if (rc != BB_OK) return rc;
    if (!bytes) return fail(BB_ERR_INVALID_ARG, "bytes is NULL");
    const int64_t b = slot_bytes(cfg, export_id);
    if (b < 0) return fail(BB_ERR_INVALID_ARG, "unknown export id " + std::to_string(export_id));
    *bytes = b;
    return BB_OK;
}

int bb_create(const bb_config *cfg, bb_sim **out) { return create_common(cfg, nullptr, 0, out); }

int bb_create_with_buffers(const bb_config *cfg, void *const *bufs, int32_t nbuf, bb_sim **out)
{
    if (!bufs) return fail(BB_ERR_INVALID_ARG, "bufs is NULL");
    return create_common(cfg, bufs, nbuf, out);
}

int bb_destroy(bb_sim *s)
{
    if (!s) return BB_OK;
    if (s->aux[0]) {
        DeviceGuard g(s->device);
        for (hipStream_t a : s->aux)
            if (a) (void)hipStreamSynchronize(a);
        for (hipEvent_t e : s->aux_ev)
            if (e) (void)hipEventDestroy(e);
        for (hipStream_t a : s->aux)
            if (a) (void)hipStreamDestroy(a);
    }
    if (s->owns) {
        for (int id = 0; id < NUM_SLOTS; id++) {
            if (!s->slot[id]) continue;
            if (s->cfg.exec_mode == BB_EXEC_CUDA) {
                DeviceGuard g(s->device);
                (void)hipFree(s->slot[id]);
            } else {
                std::free(s->slot[id]);
            }
        }
    }
    delete s;
    return BB_OK;
}

int bb_step(bb_sim *s, void *stream)
{
    if (!s) return fail(BB_ERR_INVALID_ARG, "sim is NULL");
    if (s->cfg.exec_mode == BB_EXEC_CUDA) {
        DeviceGuard g(s->device);
        hipError_t e = bb::launch_step(s->n, s->p, (hipStream_t)stream);
        if (e != hipSuccess) return hip_fail(e, "launch step kernel");
        return BB_OK;
    }
    return bb::host_step(s->n, s->p, *s->pool);
}

int bb_write_random_actions(bb_sim *s, uint32_t action_seed, uint32_t step, void *stream)
{
    if (!s) return fail(BB_ERR_INVALID_ARG, "sim is NULL");
    if (s->cfg.exec_mode == BB_EXEC_CUDA) {
        DeviceGuard g(s->device);
        hipError_t e = bb::launch_random_actions(s->n, s->p, action_seed, step, (hipStream_t)stream);
        if (e != hipSuccess) return hip_fail(e, "launch random-action kernel");
        return BB_OK;
    }
    return bb::host_random_actions(s->n, s->p, *s->pool, action_seed, step);
}

}  // extern "C"

// The hipEvent_t of a timed call (kernel_ms), destroyed on every exit.
struct EventVec {
    std::vector<hipEvent_t> ev;
    ~EventVec()
    {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
    }
    hipError_t create(size_t n)
    {
        ev.assign(n, nullptr);
        for (auto &e : ev) {
            const hipError_t r = hipEventCreate(&e);
            if (r != hipSuccess) {
                e = nullptr;
                return r;
            }
        }
        return hipSuccess;
    }
};

extern "C" {

int bb_step_n(bb_sim *s, int32_t n, int32_t random_actions, uint32_t action_seed, uint32_t step0,
              void *stream, float *kernel_ms)
{
    if (!s) return fail(BB_ERR_INVALID_ARG, "sim is NULL");
    if (n < 0) return fail(BB_ERR_INVALID_ARG, "n must be >= 0");
    if (s->cfg.exec_mode != BB_EXEC_CUDA) {
        int rc = bb::host_steps(s->n, s->p, *s->pool, n, random_actions != 0, action_seed, step0);
        if (rc != BB_OK) return rc;
        if (kernel_ms) *kernel_ms = 0.f;
        return BB_OK;
    }
    DeviceGuard g(s->device);
    hipStream_t st = (hipStream_t)stream;
    EventVec evs;
    std::vector<hipEvent_t> &ev = evs.ev;
    if (kernel_ms && n > 0) {
        const hipError_t he = evs.create((size_t)2 * n);
        if (he != hipSuccess) return hip_fail(he, "hipEventCreate");
    }
    for (int32_t k = 0; k < n; k++) {
        if (random_actions) {
            hipError_t e = bb::launch_random_actions(s->n, s->p, action_seed, step0 + (uint32_t)k, st);
            if (e != hipSuccess) return hip_fail(e, "launch random-action kernel");
        }
        // kernel_ms: the step kernel's own start/end (hipExtLaunchKernel events)
        hipError_t e = ev.empty() ? bb::launch_step(s->n, s->p, st)
                                  : bb::launch_step(s->n, s->p, st, bb::MODE_FULL, ev[2 * k], ev[2 * k + 1]);
        if (e != hipSuccess) return hip_fail(e, "launch step kernel");
    }
    if (!ev.empty()) {
        hipError_t e = hipEventSynchronize(ev.back());
        if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
        double total = 0.0;
        for (int32_t k = 0; k < n; k++) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]);
            total += ms;
        }
        *kernel_ms = (float)total;
    }
    return BB_OK;
}

int bb_fill_random_actions(bb_sim *s, int32_t *actions, int32_t n, uint32_t action_seed, uint32_t step0,
                           void *stream)
{
    if (!s || (!actions && n > 0) || n < 0) return fail(BB_ERR_INVALID_ARG, "bb_fill_random_actions");
    const int64_t rows = s->cfg.num_worlds * s->n * 6;
    bb::Params pp = s->p;
    for (int32_t k = 0; k < n; k++) {
        pp.c.action = actions + (int64_t)k * rows;
        if (s->cfg.exec_mode == BB_EXEC_CUDA) {
            DeviceGuard g(s->device);
            hipError_t e = bb::launch_random_actions(s->n, pp, action_seed, step0 + (uint32_t)k, (hipStream_t)stream);
            if (e != hipSuccess) return hip_fail(e, "launch random-action kernel");
        } else {
            int rc = bb::host_random_actions(s->n, pp, *s->pool, action_seed, step0 + (uint32_t)k);
            if (rc != BB_OK) return rc;
        }
    }
    return BB_OK;
}

// bb_step_n_staged's steps in one launch.  Kinds: 0 one k_step launch per
// step; 1 one k_step_loop launch (each wave loads the state its own lanes
// stored the step before); 2 (the 2-agent game; elsewhere 1) one k_rollout /
// k_rollout_split launch with RolloutArgs::store_state -- the state stays in
// registers between steps and every step stores all of its columns, rows,
// rewards, done flags and action write-backs where k_step does.
// Default 2 (measured faster at every size, bit-identical: 8 192 x 2 6.70 ->
// 4.93 us per step, 65 536 19.30 -> 15.76, 262 144 61.5 -> 59.8;
// profiles/r05/an_sweep.txt, ao_sweep.txt), at every agent count (the
// shared-world loop: 65 536 x 4 64.4 -> 53.6 us per step, x 10 291.7 -> 246.0,
// profiles/r05/aa_step_loop_n.txt); DIAG_STEP_LOOP forces a kind (tests, the
// bench's per-launch objects).
static int step_loop_kind()
{
    const int k = bb::diag_or(bb::DIAG_STEP_LOOP, 2);
    return k > 2 ? 2 : k;
}

// The launch bb_step_n_staged makes for n steps (BB_STAGED_*; the host
// executor: BB_STAGED_PER_STEP).  The resident loop at N >= 4 is
// k_rollout_shared's resident instance, taken while the step stays in the
// Infinity Cache (bb::resident_staged).
static int staged_path(const bb_sim *s, int32_t n)
{
    if (s->cfg.exec_mode != BB_EXEC_CUDA || n < 2) return BB_STAGED_PER_STEP;
    const int k = step_loop_kind();
    if (k == 2) return bb::resident_staged_n(s->n, s->cfg.num_worlds) ? BB_STAGED_RESIDENT : BB_STAGED_LOOP;
    return k == 1 ? BB_STAGED_LOOP : BB_STAGED_PER_STEP;
}

int32_t bb_step_staged_path(const bb_sim *s, int32_t n)
{
    if (!s || n < 0) return fail(BB_ERR_INVALID_ARG, "bb_step_staged_path");
    return staged_path(s, n);
}

int64_t bb_step_staged_bytes(const bb_sim *s, int32_t n)
{
    if (!s || n < 0) return 0;
    const int64_t B = bb_algorithmic_bytes_per_world(s->n);
    // the state reads of B(N) (120 B per agent besides its
    // action row, 120 B per world): the resident loop makes them once
    const int64_t R = 120 * ((int64_t)s->n + 1);
    const int64_t per_world = staged_path(s, n) == BB_STAGED_RESIDENT ? (int64_t)n * (B - R) + (n > 0 ? R : 0)
                                                                       : (int64_t)n * B;
    return per_world * s->cfg.num_worlds;
}

int bb_step_n_staged(bb_sim *s, int32_t n, int32_t *actions, void *stream, float *kernel_ms)
{
    if (!s || n < 0 || (!actions && n > 0)) return fail(BB_ERR_INVALID_ARG, "bb_step_n_staged");
    const int64_t rows = s->cfg.num_worlds * s->n * 6;
    bb::Params pp = s->p;
    if (s->cfg.exec_mode != BB_EXEC_CUDA) {
        for (int32_t k = 0; k < n; k++) {
            pp.c.action = actions + (int64_t)k * rows;
            int rc = bb::host_step(s->n, pp, *s->pool);
            if (rc != BB_OK) return rc;
        }
        if (n > 0) std::memcpy(s->p.c.action, actions + (int64_t)(n - 1) * rows, (size_t)rows * 4);
        if (kernel_ms) *kernel_ms = 0.f;
        return BB_OK;
    }
    DeviceGuard g(s->device);
    hipStream_t st = (hipStream_t)stream;
    // the 2-agent step: the n steps in one k_step_loop launch (each wave steps
    // its worlds n times; bit-identical to n k_step launches); otherwise, or
    // with MADRONA_BB_STEP_LOOP=0, one k_step launch per step
    const int kind = staged_path(s, n);
    const bool loop = kind != BB_STAGED_PER_STEP;
    const bool resident = kind == BB_STAGED_RESIDENT;
    EventVec evs;
    std::vector<hipEvent_t> &ev = evs.ev;
    if (kernel_ms && n > 0) {
        const hipError_t he = evs.create((size_t)2 * (loop ? 1 : n));
        if (he != hipSuccess) return hip_fail(he, "hipEventCreate");
    }
    if (resident) {
        bb::RolloutArgs r{actions, s->p.c.obs, s->p.c.reward, s->p.c.done, 0, 0, n, 1};
        hipError_t e = bb::launch_rollout(s->n, pp, r, st, ev.empty() ? nullptr : ev[0], ev.empty() ? nullptr : ev[1]);
        if (e != hipSuccess) return hip_fail(e, "launch resident step loop kernel");
    } else if (loop) {
        hipError_t e = bb::launch_step_loop(s->n, pp, actions, n, st, ev.empty() ? nullptr : ev[0],
                                            ev.empty() ? nullptr : ev[1]);
        if (e != hipSuccess) return hip_fail(e, "launch step loop kernel");
    }
    for (int32_t k = 0; k < (loop ? 0 : n); k++) {
        pp.c.action = actions + (int64_t)k * rows;
        hipError_t e = ev.empty() ? bb::launch_step(s->n, pp, st)
                                  : bb::launch_step(s->n, pp, st, bb::MODE_FULL, ev[2 * k], ev[2 * k + 1]);
        if (e != hipSuccess) return hip_fail(e, "launch step kernel");
    }
    if (n > 0 && !resident) {  // (the resident loop stores the last step's rows there itself)
        hipError_t e = hipMemcpyAsync(s->p.c.action, actions + (int64_t)(n - 1) * rows, (size_t)rows * 4,
                                      hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return hip_fail(e, "copy last actions");
    }
    if (!ev.empty()) {
        hipError_t e = hipEventSynchronize(ev.back());
        if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
        double total = 0.0;
        for (int32_t k = 0; k < (loop ? 1 : n); k++) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]);
            total += ms;
        }
        *kernel_ms = (float)total;
    }
    return BB_OK;
}

int bb_rollout(bb_sim *s, int32_t n, int32_t *actions, float *obs_out, float *reward_out, float *done_out,
               uint32_t flags, void *stream, float *kernel_ms)
{
    if (!s || n < 0 || (!actions && n > 0)) return fail(BB_ERR_INVALID_ARG, "bb_rollout");
    if (flags & ~BB_ROLLOUT_PER_STEP) return fail(BB_ERR_INVALID_ARG, "bb_rollout: unknown flag bits");
    if (kernel_ms) *kernel_ms = 0.f;
    if (n == 0) return BB_OK;
    const int64_t rows = s->cfg.num_worlds * s->n;  // [W][N]
    const int64_t ow = bb::obs_width(s->n);
    const int64_t used_bytes = (int64_t)((bb::obs_used(s->n) + 3) / 4) * 16;  // written part of a row
    bb::RolloutArgs r{};
    r.actions = actions;
    r.obs = obs_out ? obs_out : s->p.c.obs;
    r.reward = reward_out ? reward_out : s->p.c.reward;
    r.done = done_out ? done_out : s->p.c.done;
    r.obs_step = obs_out ? rows * ow : 0;
    r.rd_step = (reward_out || done_out) ? rows : 0;
    if ((reward_out == nullptr) != (done_out == nullptr))
        return fail(BB_ERR_INVALID_ARG, "bb_rollout: reward_out and done_out are recorded together");
    r.steps = n;
    const float *last_obs = r.obs + (int64_t)(n - 1) * r.obs_step;
    const float *last_rew = r.reward + (int64_t)(n - 1) * r.rd_step;
    const float *last_done = r.done + (int64_t)(n - 1) * r.rd_step;
    const int32_t *last_act = actions + (int64_t)(n - 1) * rows * 6;
    auto step_params = [&](int32_t k) {
        bb::Params pp = s->p;
        pp.c.action = actions + (int64_t)k * rows * 6;
        pp.c.obs = r.obs + (int64_t)k * r.obs_step;
        pp.c.reward = r.reward + (int64_t)k * r.rd_step;
        pp.c.done = r.done + (int64_t)k * r.rd_step;
        return pp;
    };
    if (s->cfg.exec_mode != BB_EXEC_CUDA) {
        for (int32_t k = 0; k < n; k++) {
            int rc = bb::host_step(s->n, step_params(k), *s->pool);
            if (rc != BB_OK) return rc;
        }
        std::memcpy(s->p.c.action, last_act, (size_t)rows * 24);
        if (obs_out)
            for (int64_t q = 0; q < rows; q++) std::memcpy(s->p.c.obs + q * ow, last_obs + q * ow, (size_t)used_bytes);
        if (reward_out) {
            std::memcpy(s->p.c.reward, last_rew, (size_t)rows * 4);
            std::memcpy(s->p.c.done, last_done, (size_t)rows * 4);
        }
        return BB_OK;
    }
    DeviceGuard g(s->device);
    hipStream_t st = (hipStream_t)stream;
    const bool fused = !(flags & BB_ROLLOUT_PER_STEP) && bb::fused_rollout_n(s->n);
    const int32_t launches = fused ? 1 : n;
    EventVec evs;
    std::vector<hipEvent_t> &ev = evs.ev;
    if (kernel_ms) {
        const hipError_t he = evs.create((size_t)2 * launches);
        if (he != hipSuccess) return hip_fail(he, "hipEventCreate");
    }
    hipEvent_t *evp = ev.empty() ? nullptr : ev.data();
    if (fused) {
        hipError_t e = bb::launch_rollout(s->n, s->p, r, st, evp ? evp[0] : nullptr, evp ? evp[1] : nullptr);
        if (e != hipSuccess) return hip_fail(e, "launch rollout kernel");
    } else {
        for (int32_t k = 0; k < n; k++) {
            hipError_t e = bb::launch_step(s->n, step_params(k), st, bb::MODE_FULL, evp ? evp[2 * k] : nullptr,
                                           evp ? evp[2 * k + 1] : nullptr);
            if (e != hipSuccess) return hip_fail(e, "launch step kernel");
        }
        hipError_t e = hipMemcpyAsync(s->p.c.action, last_act, (size_t)rows * 24, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return hip_fail(e, "copy last actions");
        if (reward_out) {
            e = hipMemcpyAsync(s->p.c.reward, last_rew, (size_t)rows * 4, hipMemcpyDeviceToDevice, st);
            if (e == hipSuccess) e = hipMemcpyAsync(s->p.c.done, last_done, (size_t)rows * 4, hipMemcpyDeviceToDevice, st);
            if (e != hipSuccess) return hip_fail(e, "copy last reward/done");
        }
    }
    // the written part of every row (the zero tail stays); the N = 2 rollout
    // kernels store the last step's rows into the sim's tensor themselves (at
    // N >= 4 that second store made every step of k_rollout_shared slower:
    // 1 470 -> 1 677 us per 32-step launch, against a copy of ~200 us)
    if (obs_out && !(fused && s->n == 2)) {
        hipError_t e = hipMemcpy2DAsync(s->p.c.obs, (size_t)ow * 4, last_obs, (size_t)ow * 4, (size_t)used_bytes,
                                        (size_t)rows, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return hip_fail(e, "copy last observations");
    }
    if (!ev.empty()) {
        hipError_t e = hipEventSynchronize(ev.back());
        if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
        double total = 0.0;
        for (int32_t k = 0; k < launches; k++) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]);
            total += ms;
        }
        *kernel_ms = (float)total;
    }
    return BB_OK;
}

int bb_policy_forward(const bb_policy_weights *w, int32_t exec_mode, int32_t gpu_id, const float *obs, int64_t rows,
                      int64_t obs_stride, int32_t *actions, int64_t action_stride, float *log_prob, float *value,
                      int32_t stochastic, uint32_t seed, uint32_t step, void *stream)
{
    if (!w || !obs || !actions || rows < 0 || obs_stride < bb::POL_IN || action_stride < 6)
        return fail(BB_ERR_INVALID_ARG, "bb_policy_forward: arguments");
    const float *req[] = {w->obs_mean, w->obs_inv, w->w1, w->b1, w->ln1_w, w->ln1_b, w->w2, w->b2, w->ln2_w,
                          w->ln2_b, w->head_w, w->head_b};
    for (const float *ptr : req)
        if (!ptr) return fail(BB_ERR_INVALID_ARG, "bb_policy_forward: a weight pointer is NULL");
    if ((((uintptr_t)obs) & 15u) || (obs_stride & 3) || (((uintptr_t)w->w1) & 15u))
        return fail(BB_ERR_INVALID_ARG, "bb_policy_forward: obs rows and w1 must be 16-byte aligned");
    bb::PolicyArgs a{};
    a.w = bb::PolicyWeights{w->obs_mean, w->obs_inv, w->w1, w->b1, w->ln1_w, w->ln1_b,
                            w->w2, w->b2, w->ln2_w, w->ln2_b, w->head_w, w->head_b};
    a.obs = obs; a.obs_stride = obs_stride; a.rows = rows;
    a.actions = actions; a.act_stride = action_stride;
    a.log_prob = log_prob; a.value = value;
    a.stochastic = stochastic ? 1 : 0; a.seed = seed; a.step = step;
    if (exec_mode == BB_EXEC_CPU) {
        bb::host_policy(a);
        return BB_OK;
    }
    if (exec_mode != BB_EXEC_CUDA) return fail(BB_ERR_INVALID_ARG, "bb_policy_forward: exec_mode");
    DeviceGuard g(gpu_id);
    hipError_t e = bb::launch_policy(a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "launch policy kernel");
    return BB_OK;
}

namespace {

// Start / end events of a timed region, destroyed on every exit path.
struct EventPair {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    bool create() { return hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess; }
    ~EventPair()
    {
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
    }
};

bool weights_ok(const bb_policy_weights *w)
{
    if (!w) return false;
    const float *req[] = {w->obs_mean, w->obs_inv, w->w1, w->b1, w->ln1_w, w->ln1_b, w->w2, w->b2, w->ln2_w,
                          w->ln2_b, w->head_w, w->head_b};
    for (const float *ptr : req)
        if (!ptr) return false;
    return (((uintptr_t)w->w1) & 15u) == 0;
}

bb::PolicyWeights policy_weights(const bb_policy_weights *w)
{
    return bb::PolicyWeights{w->obs_mean, w->obs_inv, w->w1, w->b1, w->ln1_w, w->ln1_b,
                             w->w2, w->b2, w->ln2_w, w->ln2_b, w->head_w, w->head_b};
}

}  // namespace

// Params of worlds [w0, w0 + count) of a simulator: every column advanced by
// w0 worlds, world_offset (the per-world RNG key) too, so the part steps
// exactly as those worlds of the whole (the worlds are independent).
bb::Params shard_params(const bb::Params &p, int N, int64_t w0, int64_t count)
{
    bb::Params q = p;
    bb::Columns &c = q.c;
    const auto off = [&](auto *&ptr, int64_t per_world) {
        if (ptr) ptr += w0 * per_world;
    };
    off(c.reset, N); off(c.game_state, 14); off(c.action, N * 6); off(c.action_mask, N * 4);
    off(c.agent_pos, N * 3); off(c.obs, N * bb::obs_width(N)); off(c.reward, N); off(c.done, N);
    off(c.agent_id, N); off(c.possession, N * 3); off(c.orientation, N * 4); off(c.team, N * 5);
    off(c.stats, N * 2); off(c.ball_pos, 3); off(c.ball_physics, 7); off(c.ball_id, 1); off(c.ball_grabbed, 2);
    off(c.ball_vel, 3); off(c.hoop_pos, 6); off(c.agent_vel, N * 3); off(c.cooldown, N); off(c.cur_step, N);
    off(c.inbounding, N * 2); off(c.attributes, N * 10); off(c.world_clock, 1); off(c.rng_counter, 1);
    q.num_worlds = count;
    q.world_offset = p.world_offset + w0;
    return q;
}

// Split per-step PPO loop (bb_rollout_policy) from this many worlds on: the
// two halves of the worlds run on two streams, half B's first policy pass
// after half A's, so one half's policy pass (latency-bound) runs beside the
// other half's step (memory-bound).  The halves' policy passes take
// k_policy<2> (256 VGPRs + 19 AGPRs: a policy wave and a 224-VGPR step wave
// share a SIMD's 512; k_policy<4>'s 256 + 220 do not, and then the kernels
// only alternate: 58.9 us per step at 65 536 worlds).  Measured per step,
// K = 32, all records (profiles/r04/r_*, v_*, z_*): 32 768 worlds 41.0 ->
// 35.4 us, 65 536 56.1 -> 50.1-51.3 (k_policy<1> halves 51.9-53.2,
// k_policy_wg 54.7-55.5), 131 072 99.5 -> 92.5, 262 144 187.2 -> 176.4.
// The parts are independent worlds, so nothing orders them but the start:
// part h's first policy pass waits for part h - 1's (re-aligning them every
// step, an event per step, measured 54.5-55.7 vs 52.3-53.5 us per step,
// profiles/r04/v_*).  The parts' policy kernel is k_policy<2> (276 registers:
// a policy wave fits beside a step wave on one SIMD).
constexpr int64_t PPO_SPLIT_MIN_WORLDS = 32768;
constexpr int PPO_SPLIT_PARTS = 2;
constexpr int PPO_SPLIT_MT = 2;

// The fused PPO rollout (k_rollout_policy) runs one workgroup of 3 waves per
// 32 worlds at one workgroup per CU (register-bound): used up to two waves of
// workgroups -- measured 8 192 worlds 15.1 vs 27.6 us per step unfused,
// 16 384: 29.7 vs 33.4, 65 536: 115 vs 64 (profiles/r03/g_ppo_fused_ab.txt).
// DIAG_PPO_FUSED_MAX_WORLDS overrides the bound (tests).
static int64_t ppo_fused_max_worlds() { return bb::diag_or(bb::DIAG_PPO_FUSED_MAX_WORLDS, 16384); }

// The fused step's rollout as one k_rollout_ppo launch (default) or as one
// k_step_ppo launch per step (DIAG_PPO_STEP_LOOP = 0; bit-identical, tests).
static bool ppo_step_loop() { return bb::diag_or(bb::DIAG_PPO_STEP_LOOP, 1) != 0; }

// PPO's loop with the trainee's policy pass fused behind the world step (its
// rows read from LDS; k_rollout_ppo) from this many worlds on, wherever the
// register-resident k_rollout_policy (<= 16 384 worlds) is not taken:
// measured 24 576 worlds 31.2 -> 20.0 us per step against the two-stream
// split, while at 8 192 / 16 384 k_rollout_policy stays ahead (10.1 / 12.4 vs
// 18.2 / 19.2; profiles/r05/k_small_ab.txt).
// DIAG_PPO_STEP_FUSED_MIN_WORLDS overrides it (0: never; tests).
static int64_t ppo_step_fused_min_worlds() { return bb::diag_or(bb::DIAG_PPO_STEP_FUSED_MIN_WORLDS, 1); }

// The implementation bb_rollout_policy takes (BB_PPO_PATH_*).
static int32_t ppo_path(const bb_sim *s, bool opponent, uint32_t flags)
{
    if (s->cfg.exec_mode != BB_EXEC_CUDA) return BB_PPO_PATH_HOST;
    if (s->n != 2) return -1;  // bb_rollout_policy: the reference's 2-agent game only
    const int64_t W = s->cfg.num_worlds;
    if (!(flags & BB_ROLLOUT_PER_STEP) && !opponent && bb::fused_rollout_n(s->n) && W <= ppo_fused_max_worlds())
        return BB_PPO_PATH_FUSED_ROLLOUT;
    if (!(flags & BB_ROLLOUT_PER_STEP) && !opponent && s->n == 2 && ppo_step_fused_min_worlds() > 0 &&
        W >= ppo_step_fused_min_worlds())
        return BB_PPO_PATH_FUSED_STEP;
    return BB_PPO_PATH_PER_STEP;
}

int bb_rollout_policy(bb_sim *s, const bb_policy_weights *w, const bb_policy_weights *opponent, int32_t n,
                      int32_t trainee, int32_t stochastic, uint32_t seed, uint32_t step0,
                      const bb_policy_rollout_buffers *out, uint32_t flags, void *stream, float *kernel_ms)
{
    if (flags & ~BB_ROLLOUT_PER_STEP) return fail(BB_ERR_INVALID_ARG, "bb_rollout_policy: unknown flag bits");
    if (!s || n < 0 || !out) return fail(BB_ERR_INVALID_ARG, "bb_rollout_policy: arguments");
    if (kernel_ms) *kernel_ms = 0.f;
    if (!weights_ok(w) || (opponent && !weights_ok(opponent)))
        return fail(BB_ERR_INVALID_ARG, "bb_rollout_policy: a weight pointer is NULL or w1 is not 16-byte aligned");
    if (s->n != 2) return fail(BB_ERR_UNSUPPORTED, "bb_rollout_policy: the reference's 2-agent game only");
    if (trainee < 0 || trainee >= s->n) return fail(BB_ERR_INVALID_ARG, "bb_rollout_policy: trainee index");
    if (n == 0) return BB_OK;
    if ((out->reward == nullptr) != (out->done == nullptr))
        return fail(BB_ERR_INVALID_ARG, "bb_rollout_policy: reward and done are recorded together");
    const int64_t W = s->cfg.num_worlds, N = s->n, ow = bb::obs_width(s->n);
    const bb::Columns &c = s->p.c;
    // Per step k (scripts/ppo.py:65-134 over scripts/env.py:126-170):
    //   actions, log_probs, values = agent(obs)       policy on the trainee rows
    //   [frozen opponent acts, env.py:127-143]        policy on the other rows
    //   actions[:, trainee] = a; worlds.step()         env.py:147,155
    //   buffer.{obs, actions, log_probs, values}[k]    recorded by the policy pass
    //   buffer.{rewards, not_dones}[k]                 recorded by the next pass
    // and after the last step next_value = agent.evaluate(obs_) (ppo.py:136-137),
    // a value-only pass that also records step n-1's rewards / dones.
    auto pass = [&](int32_t k, bool final_pass) {
        bb::PolicyArgs a{};
        a.w = policy_weights(w);
        a.obs = c.obs + trainee * ow; a.obs_stride = N * ow; a.rows = W;
        a.stochastic = stochastic ? 1 : 0; a.seed = seed; a.step = step0 + (uint32_t)k;
        if (!final_pass) {
            a.actions = c.action + trainee * 6; a.act_stride = N * 6;
            a.obs_out = out->obs ? out->obs + (int64_t)k * W * bb::POL_IN : nullptr;
            a.act_out = out->actions ? out->actions + (int64_t)k * W * 6 : nullptr;
            a.log_prob = out->log_prob ? out->log_prob + (int64_t)k * W : nullptr;
            a.value = out->value ? out->value + (int64_t)k * W : nullptr;
        } else {
            a.value = out->next_value;
        }
        if (k > 0 && out->reward) {
            a.rew_src = c.reward + trainee; a.done_src = c.done + trainee; a.rd_stride = N;
            a.rew_out = out->reward + (int64_t)(k - 1) * W;
            a.done_out = out->done + (int64_t)(k - 1) * W;
        }
        return a;
    };
    auto opp_pass = [&](int32_t k) {
        bb::PolicyArgs a{};
        a.w = policy_weights(opponent);
        const int other = 1 - trainee;
        a.obs = c.obs + other * ow; a.obs_stride = N * ow; a.rows = W;
        a.actions = c.action + other * 6; a.act_stride = N * 6;
        // the frozen policy samples (Agent.forward's default) with its own key
        a.stochastic = 1; a.seed = seed ^ 0x9E3779B9u; a.step = step0 + (uint32_t)k;
        return a;
    };
    const bool final_needed = out->next_value != nullptr || out->reward != nullptr;
    if (s->cfg.exec_mode != BB_EXEC_CUDA) {
        for (int32_t k = 0; k < n; k++) {
            bb::host_policy(pass(k, false));
            if (opponent) bb::host_policy(opp_pass(k));
            int rc = bb::host_step(s->n, s->p, *s->pool);
            if (rc != BB_OK) return rc;
        }
        if (final_needed) bb::host_policy(pass(n, true));
        return BB_OK;
    }
    // the kernels store obs rows as float4 and action rows as int2
    const auto misaligned = [](const void *ptr, uintptr_t a) { return ptr && ((uintptr_t)ptr & (a - 1)) != 0; };
    if (misaligned(out->obs, 16) || misaligned(out->actions, 8))
        return fail(BB_ERR_INVALID_ARG, "bb_rollout_policy: out->obs must be 16-byte and out->actions 8-byte aligned");
    DeviceGuard g(s->device);
    hipStream_t st = (hipStream_t)stream;
    EventPair ev;  // destroyed on every exit
    if (kernel_ms) {
        if (!ev.create()) return fail(BB_ERR_HIP, "hipEventCreate");
        (void)hipEventRecord(ev.e0, st);
    }
    const int32_t path = ppo_path(s, opponent != nullptr, flags);
    const bool fused = path == BB_PPO_PATH_FUSED_ROLLOUT;
    if (fused) {
        bb::PolicyRolloutArgs r{};
        r.w = policy_weights(w);
        r.obs_out = out->obs; r.act_out = out->actions; r.log_prob = out->log_prob; r.value = out->value;
        r.reward = out->reward; r.done = out->done; r.next_value = out->next_value;
        r.steps = n; r.trainee = trainee; r.stochastic = stochastic ? 1 : 0; r.seed = seed; r.step0 = step0;
        hipError_t e = bb::launch_rollout_policy(s->n, s->p, r, st);
        if (e != hipSuccess) return hip_fail(e, "launch fused PPO rollout kernel");
    }
    const bool step_fused = path == BB_PPO_PATH_FUSED_STEP;
    if (step_fused) {
        // policy pass 0 on the sim's rows, then per step k one k_step_ppo:
        // step k, then policy pass k + 1 (or the value pass after the last step)
        // (the k_step_ppo launches need the policy pass of step 0 before them;
        // k_rollout_ppo runs it itself)
        const bool in_kernel = ppo_step_loop();
        hipError_t e = in_kernel ? hipSuccess : bb::launch_policy(pass(0, false), st);
        if (e == hipSuccess && ppo_step_loop()) {
            // the whole rollout in one k_rollout_ppo launch
            bb::PpoStepArgs a{};
            a.pass0 = in_kernel ? 1 : 0;
            a.step0 = step0;
            a.obs0 = out->obs;
            a.act0 = out->actions;
            a.log_prob0 = out->log_prob;
            a.value0 = out->value;
            a.w = policy_weights(w);
            a.trainee = trainee; a.stochastic = stochastic ? 1 : 0; a.seed = seed;
            a.step = step0 + 1u;
            a.reward = out->reward;
            a.done = out->done;
            if (n > 1) {
                a.obs_rec = out->obs ? out->obs + W * bb::POL_IN : nullptr;
                a.act_out = out->actions ? out->actions + W * 6 : nullptr;
                a.log_prob = out->log_prob ? out->log_prob + W : nullptr;
                a.value = out->value ? out->value + W : nullptr;
            }
            a.value_last = out->next_value;
            e = bb::launch_rollout_ppo(s->n, s->p, a, n, st);
        }
        for (int32_t k = 0; k < (ppo_step_loop() ? 0 : n) && e == hipSuccess; k++) {
            bb::PpoStepArgs a{};
            a.w = policy_weights(w);
            a.trainee = trainee; a.stochastic = stochastic ? 1 : 0; a.seed = seed;
            a.step = step0 + (uint32_t)(k + 1);
            a.last = k + 1 == n ? 1 : 0;
            if (out->reward) {
                a.reward = out->reward + (int64_t)k * W;
                a.done = out->done + (int64_t)k * W;
            }
            if (!a.last) {
                const int64_t k1 = k + 1;
                a.obs_rec = out->obs ? out->obs + k1 * W * bb::POL_IN : nullptr;
                a.act_out = out->actions ? out->actions + k1 * W * 6 : nullptr;
                a.log_prob = out->log_prob ? out->log_prob + k1 * W : nullptr;
                a.value = out->value ? out->value + k1 * W : nullptr;
            } else {
                a.value = out->next_value;
            }
            e = bb::launch_step_ppo(s->n, s->p, a, st);
        }
        if (e != hipSuccess) return hip_fail(e, "bb_rollout_policy fused step launch");
    }
    // one part (worlds [w0, w0 + cnt)) of policy pass k (or of the opponent's)
    const auto part_pass = [&](bb::PolicyArgs a, int64_t w0, int64_t cnt, const bb::Params &sp) {
        const auto adv = [&](auto *&ptr, int64_t per) {
            if (ptr) ptr += w0 * per;
        };
        a.obs += w0 * a.obs_stride;
        a.rows = cnt;
        adv(a.actions, N * 6);
        adv(a.obs_out, bb::POL_IN);
        adv(a.act_out, 6);
        adv(a.log_prob, 1);
        adv(a.value, 1);
        if (a.rew_src) {
            a.rew_src = sp.c.reward + (a.rew_src - c.reward);
            a.done_src = sp.c.done + (a.done_src - c.done);
            adv(a.rew_out, 1);
            adv(a.done_out, 1);
        }
        a.key_row0 = (uint32_t)w0;
        a.mt = PPO_SPLIT_MT;
        return a;
    };
    // the split needs at least 32 worlds (one policy tile) per part
    const bool split = !fused && !step_fused && W >= PPO_SPLIT_MIN_WORLDS && W >= 32 * (int64_t)PPO_SPLIT_PARTS;
    // steps 0 .. n-2 write the trainee's rows into buffer.obs[k + 1] only (the
    // sim's copy of them is read by nobody before the last step rewrites
    // every row); the next policy pass reads them there.  Only the agent-lane
    // step kernel records (bb::step_records); elsewhere the policy pass keeps
    // the record and reads the sim's rows.
    const bool step_rec = bb::step_records(s->n);
    const bool rec_only = out->obs != nullptr && step_rec;
    const int parts = split ? PPO_SPLIT_PARTS : 1;
    constexpr int MP = bb_sim::MAX_PARTS;
    hipStream_t pst[MP] = {st, st, st, st};
    if (split) {
        if (!s->aux[0]) {
            // all streams and events or none: created into locals, committed together
            hipStream_t as[MP - 1] = {};
            hipEvent_t ae[2 * MP] = {};
            bool ok = true;
            for (hipStream_t &a : as) ok = ok && hipStreamCreateWithFlags(&a, hipStreamNonBlocking) == hipSuccess;
            for (hipEvent_t &e : ae) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
            if (!ok) {
                for (hipStream_t a : as)
                    if (a) (void)hipStreamDestroy(a);
                for (hipEvent_t e : ae)
                    if (e) (void)hipEventDestroy(e);
                return fail(BB_ERR_HIP, "bb_rollout_policy: creating the split's streams / events");
            }
            for (int i = 0; i < MP - 1; i++) s->aux[i] = as[i];
            for (int i = 0; i < 2 * MP; i++) s->aux_ev[i] = ae[i];
        }
        // every part starts after everything before the call on the caller's stream
        hipError_t e = hipEventRecord(s->aux_ev[0], st);
        for (int h = 1; h < parts && e == hipSuccess; h++) {
            pst[h] = s->aux[h - 1];
            e = hipStreamWaitEvent(pst[h], s->aux_ev[0], 0);
        }
        if (e != hipSuccess) return hip_fail(e, "bb_rollout_policy split start");
    }
    // the caller's stream continues after every part's work -- also after an
    // error, so that nothing still queued on a part's stream outlives the call
    // unordered (the caller may free or reuse the buffers it writes)
    const auto join = [&]() -> hipError_t {
        hipError_t first = hipSuccess;
        for (int h = 1; h < parts; h++) {
            hipError_t e = hipEventRecord(s->aux_ev[MP + h], pst[h]);
            if (e == hipSuccess) e = hipStreamWaitEvent(st, s->aux_ev[MP + h], 0);
            if (e != hipSuccess) e = hipStreamSynchronize(pst[h]);  // ordered the hard way
            if (first == hipSuccess) first = e;
        }
        return first;
    };
    bb::Params sp[MP];
    int64_t pw0[MP], pcnt[MP];
    for (int h = 0; h < parts; h++) {
        pw0[h] = W * h / parts;
        pcnt[h] = W * (h + 1) / parts - pw0[h];
        sp[h] = split ? shard_params(s->p, s->n, pw0[h], pcnt[h]) : s->p;
    }
    // buffer.obs[k + 1] (the trainee's rows after step k) is written by step
    // k's row passes as whole-line stores (Params::rec_obs), so policy pass
    // k >= 1 reads its rows without recording them: from the policy's
    // registers the record took 9 us of a 61.6 us step at 65 536 worlds
    // (each store instruction touching 64 rows' lines; profiles/r04/h_*)
    for (int32_t k = 0; k < ((fused || step_fused) ? 0 : n); k++) {
        for (int h = 0; h < parts; h++) {
            bb::PolicyArgs a = pass(k, false);
            if (k > 0) a.obs_out = nullptr;
            if (k > 0 && rec_only) {  // the rows step k - 1 wrote into buffer.obs[k] only
                a.obs = out->obs + (int64_t)k * W * bb::POL_IN;
                a.obs_stride = bb::POL_IN;
            }
            if (split) a = part_pass(a, pw0[h], pcnt[h], sp[h]);
            hipError_t e = bb::launch_policy(a, pst[h]);
            if (e == hipSuccess && opponent) {
                bb::PolicyArgs o = opp_pass(k);
                if (split) o = part_pass(o, pw0[h], pcnt[h], sp[h]);
                e = bb::launch_policy(o, pst[h]);
            }
            if (e == hipSuccess && split && h + 1 < parts && k == 0) {
                // part h + 1's policy pass k starts when part h's has finished:
                // it then runs beside part h's step
                e = hipEventRecord(s->aux_ev[1 + h], pst[h]);
                if (e == hipSuccess) e = hipStreamWaitEvent(pst[h + 1], s->aux_ev[1 + h], 0);
            }
            if (e == hipSuccess) {
                bb::Params p = sp[h];
                if (out->obs && k + 1 < n && step_rec) {
                    p.rec_obs = out->obs + (int64_t)(k + 1) * W * bb::POL_IN + pw0[h] * bb::POL_IN;
                    p.rec_agent = trainee;
                    p.rec_only = rec_only ? 1 : 0;
                }
                e = bb::launch_step(s->n, p, pst[h]);
            }
            if (e != hipSuccess) {
                (void)join();
                return hip_fail(e, "bb_rollout_policy launch");
            }
        }
    }
    if (final_needed && split) {  // each part's value pass on its own stream, beside the others' last steps
        for (int h = 0; h < parts; h++) {
            hipError_t e = bb::launch_policy(part_pass(pass(n, true), pw0[h], pcnt[h], sp[h]), pst[h]);
            if (e != hipSuccess) {
                (void)join();
                return hip_fail(e, "bb_rollout_policy final pass");
            }
        }
    }
    {
        const hipError_t e = join();
        if (e != hipSuccess) return hip_fail(e, "bb_rollout_policy join");
    }
    if (final_needed && !fused && !split && !step_fused) {
        hipError_t e = bb::launch_policy(pass(n, true), st);
        if (e != hipSuccess) return hip_fail(e, "bb_rollout_policy final pass");
    }
    if (kernel_ms) {
        (void)hipEventRecord(ev.e1, st);
        hipError_t e = hipEventSynchronize(ev.e1);
        float ms = 0.f;
        if (e == hipSuccess) (void)hipEventElapsedTime(&ms, ev.e0, ev.e1);
        if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
        *kernel_ms = ms;
    }
    return BB_OK;
}

int32_t bb_record_words(int32_t n) { return bb::record_words(n); }

int bb_record(bb_sim *s, int64_t world0, int32_t count, int32_t *dst, int64_t slot, void *stream)
{
    if (!s || !dst || count < 0 || slot < 0) return fail(BB_ERR_INVALID_ARG, "bb_record");
    if (world0 < 0 || world0 + count > s->cfg.num_worlds)
        return fail(BB_ERR_INVALID_ARG, "bb_record: worlds [" + std::to_string(world0) + ", " +
                                            std::to_string(world0 + count) + ") outside the simulator");
    const bb::RecordArgs a = bb::record_args(s->p, s->n);
    uint32_t *d = (uint32_t *)dst + slot * (int64_t)count * bb::record_words(s->n);
    if (s->cfg.exec_mode != BB_EXEC_CUDA) {
        bb::host_record(a, world0, count, d);
        return BB_OK;
    }
    DeviceGuard g(s->device);
    hipError_t e = bb::launch_record(a, world0, count, d, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "launch record kernel");
    return BB_OK;
}

int bb_set_action(bb_sim *s, int32_t world_idx, int32_t agent_idx, int32_t move_speed, int32_t move_angle,
                  int32_t rotate, int32_t grab, int32_t pass, int32_t shoot, void *stream)
{
    if (!s) return fail(BB_ERR_INVALID_ARG, "sim is NULL");
    if (world_idx < 0 || world_idx >= s->cfg.num_worlds || agent_idx < 0 || agent_idx >= s->n) {
        char msg[160];
        std::snprintf(msg, sizeof(msg), "Invalid indices! world=%d (max=%lld), agent=%d (max=%d)", world_idx,
                      (long long)s->cfg.num_worlds - 1, agent_idx, s->n - 1);
        return fail(BB_ERR_INVALID_ARG, msg);
    }
    const int32_t vals[6] = {move_speed, move_angle, rotate, grab, pass, shoot};
    int32_t *dst = s->p.c.action + ((int64_t)world_idx * s->n + agent_idx) * 6;
    if (s->cfg.exec_mode == BB_EXEC_CUDA) {
        DeviceGuard g(s->device);
        hipError_t e = bb::launch_poke(dst, 6, vals, (hipStream_t)stream);
        if (e != hipSuccess) return hip_fail(e, "set_action");
        return BB_OK;
    }
    std::memcpy(dst, vals, sizeof(vals));
    return BB_OK;
}

int bb_trigger_reset(bb_sim *s, int32_t world_idx, void *stream)
{
    if (!s) return fail(BB_ERR_INVALID_ARG, "sim is NULL");
    // src/mgr.cpp:303: an out-of-range world is silently ignored
    if (world_idx < 0 || world_idx >= s->cfg.num_worlds) return BB_OK;
    int32_t *dst = s->p.c.reset + (int64_t)world_idx * s->n;
    int32_t vals[8];
    for (int k = 0; k < 8; k++) vals[k] = 1;
    if (s->cfg.exec_mode == BB_EXEC_CUDA) {
        DeviceGuard g(s->device);
        hipError_t e = bb::launch_poke(dst, s->n, vals, (hipStream_t)stream);
        if (e != hipSuccess) return hip_fail(e, "trigger_reset");
        return BB_OK;
    }
    for (int k = 0; k < s->n; k++) dst[k] = 1;
    return BB_OK;
}

int bb_export(bb_sim *s, int32_t export_id, void **ptr, int32_t *dtype, int32_t *ndim, int64_t dims[4])
{
    if (!s) return fail(BB_ERR_INVALID_ARG, "sim is NULL");
    if (!slot_used(export_id)) return fail(BB_ERR_INVALID_ARG, "unknown export id " + std::to_string(export_id));
    if (!export_info(export_id, s->n, s->cfg.num_worlds, dtype, ndim, dims, nullptr))
        return fail(BB_ERR_INVALID_ARG, "unknown export id");
    if (ptr) *ptr = s->slot[export_id];
    return BB_OK;
}

int64_t bb_num_worlds(const bb_sim *s) { return s ? s->cfg.num_worlds : 0; }
int32_t bb_num_agents(const bb_sim *s) { return s ? s->n : 0; }
int32_t bb_exec_mode(const bb_sim *s) { return s ? s->cfg.exec_mode : -1; }

// Diagnostic (not in the public header): bb_step_n_staged's steps as one
// register-resident rollout launch (2), one k_step_loop launch (1), one
// k_step launch per step (0) or by the environment (-1) for the calls that
// follow (bench's per-launch object, A/B tests).
int bb_diag_step_loop(int32_t v)
{
    if (v < -1 || v > 2) return fail(BB_ERR_INVALID_ARG, "bb_diag_step_loop: -1, 0, 1 or 2");
    bb::diag_override[bb::DIAG_STEP_LOOP] = v;
    return BB_OK;
}

// Diagnostic (not in the public header): k_rollout_split on (1), off (0) or
// by grid size (-1) for the rollouts that follow (bit-parity tests of both).
int bb_diag_force_rollout_split(int32_t v)
{
    if (v < -1 || v > 1) return fail(BB_ERR_INVALID_ARG, "bb_diag_force_rollout_split: -1, 0 or 1");
    bb::diag_override[bb::DIAG_ROLLOUT_SPLIT] = v;
    return BB_OK;
}

// Diagnostic (not in the public header): the kernel a call launches, as
// rocprofv3 names it (without the parameter list) -- what = 0: bb_step; 1:
// bb_step_n_staged of n steps; 2: bb_rollout of n steps.  From the same
// selection rules the launchers use (bench.py labels its lines with it).
const char *bb_diag_kernel_name(const bb_sim *s, int32_t what, int32_t n)
{
    static thread_local std::string name;
    if (!s || s->cfg.exec_mode != BB_EXEC_CUDA) return "";
    const std::string N = std::to_string(s->n);
    const auto rollout = [&](bool store) -> std::string {
        switch (bb::rollout_kernel_n(s->n, s->cfg.num_worlds)) {
        case bb::RK_SPLIT: return "bb::k_rollout_split<" + N + (store ? ", true>" : ">");
        case bb::RK_MINW1: return "bb::k_rollout<" + N + (store ? ", 1, 1, true>" : ", 1>");
        case bb::RK_MINW2: return "bb::k_rollout<" + N + (store ? ", 2, 1, true>" : ", 2>");
        case bb::RK_SHARED: return "bb::k_rollout_shared<" + N + (store ? ", true>" : ">");
        default: return "bb::k_step<" + N + ">";
        }
    };
    if (what == 1) {
        const int path = staged_path(s, n);
        name = path == BB_STAGED_RESIDENT ? rollout(true)
             : path == BB_STAGED_LOOP     ? "bb::k_step_loop<" + N + ">"
                                          : "bb::k_step<" + N + ">";
    } else if (what == 2) {
        name = bb::fused_rollout_n(s->n) ? rollout(false) : "bb::k_step<" + N + ">";
    } else {
        name = "bb::k_step<" + N + ">";
    }
    return name.c_str();
}

// Diagnostic (not in the public header): a path override of bb_launch.h's
// DiagKey table for the calls that follow (-1: the product's own rule).  The
// only way to change a launch choice: nothing is read from the environment.
int bb_diag_set(int32_t key, int32_t value)
{
    if (key < 0 || key >= bb::DIAG_KEYS || value < -1) return fail(BB_ERR_INVALID_ARG, "bb_diag_set: key / value");
    bb::diag_override[key] = value;
    return BB_OK;
}

// Diagnostic (not in the public header): average ms of `iters` back-to-back
// launches of a k_step variant (bb::StepMode) or, for mode 100, of a
// coalesced streaming probe moving read_q/write_q 16-byte pieces per world.
int bb_diag_time(bb_sim *s, int32_t mode, int32_t iters, int32_t read_q, int32_t write_q, void *stream,
                 float *avg_ms)
{
    // MODE_SKIP (5): read_q carries the skip mask (Params::diag_skip), write_q
    // the run-twice mask (Params::diag_dup)
    const uint32_t skip = (mode == 5) ? (uint32_t)read_q : 0u;
    const uint32_t dup = (mode == 5) ? (uint32_t)write_q : 0u;
    if (!s || s->cfg.exec_mode != BB_EXEC_CUDA || iters < 1 || !avg_ms) return fail(BB_ERR_INVALID_ARG, "bb_diag_time");
    DeviceGuard g(s->device);
    hipStream_t st = (hipStream_t)stream;
    float4 *src = nullptr, *dst = nullptr;
    const int64_t W = s->cfg.num_worlds;
    const bool probe = mode >= 100 && mode <= 103;  // 100 + 2*nt + region pattern
    if (probe) {
        if (hipMalloc(&src, (size_t)W * read_q * 16) != hipSuccess || hipMalloc(&dst, (size_t)W * write_q * 16) != hipSuccess)
            return fail(BB_ERR_OOM, "probe buffers");
        (void)hipMemsetAsync(src, 0, (size_t)W * read_q * 16, st);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    bb::Params pp = s->p;
    pp.diag_skip = skip;
    pp.diag_dup = dup;
    pp.diag_keep = 0;
    auto once = [&]() -> hipError_t {
        if (probe) return bb::launch_stream_probe(src, dst, W, read_q, write_q, (mode - 100) & 1, (mode - 100) >> 1, st);
        return bb::launch_step(s->n, pp, st, mode);
    };
    hipError_t e = once();  // warm
    if (e == hipSuccess) {
        (void)hipEventRecord(e0, st);
        for (int k = 0; k < iters && e == hipSuccess; k++) e = once();
        (void)hipEventRecord(e1, st);
        (void)hipEventSynchronize(e1);
    }
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (src) (void)hipFree(src);
    if (dst) (void)hipFree(dst);
    if (e != hipSuccess) return hip_fail(e, "diag launch");
    *avg_ms = ms / iters;
    return BB_OK;
}

// Diagnostic (not in the public header): one MODE_TRACE launch; copies the
// per-wave phase clocks and reset-lane count (bb_kernels.hip TRACE_POINTS)
// into out[waves][12].  *waves = number of waves of the launch.
int bb_diag_trace(bb_sim *s, void *stream, uint64_t *out, int64_t max_waves, int64_t *waves)
{
    if (!s || s->cfg.exec_mode != BB_EXEC_CUDA || !out || !waves) return fail(BB_ERR_INVALID_ARG, "bb_diag_trace");
    DeviceGuard g(s->device);
    hipStream_t st = (hipStream_t)stream;
    const int64_t nw = bb::step_grid_n(s->n, s->cfg.num_worlds);
    *waves = nw;
    if (nw > max_waves) return fail(BB_ERR_INVALID_ARG, "bb_diag_trace: out too small");
    bb::Params pp = s->p;
    if (hipMalloc(&pp.diag_ts, (size_t)nw * 12 * sizeof(uint64_t)) != hipSuccess) return fail(BB_ERR_OOM, "trace buffer");
    hipError_t e = bb::launch_step(s->n, pp, st, bb::MODE_TRACE);  // warm
    if (e == hipSuccess) e = bb::launch_step(s->n, pp, st, bb::MODE_TRACE);
    if (e == hipSuccess) e = hipMemcpyAsync(out, pp.diag_ts, (size_t)nw * 12 * sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(pp.diag_ts);
    if (e != hipSuccess) return hip_fail(e, "diag trace");
    return BB_OK;
}

// Diagnostic (not in the public header): out[i] = f(x[i]) (or f(x[i], y[i]))
// of the step's scalar math on the device (bb_common.hip k_math_probe), for
// bit-for-bit comparison with the host build of bb_math.h.
int bb_diag_math(int32_t fn, const float *x, const float *y, float *out, int64_t n, int32_t gpu_id, void *stream)
{
    if (!x || !out || n < 0 || (fn == 4 && !y)) return fail(BB_ERR_INVALID_ARG, "bb_diag_math");
    DeviceGuard g(gpu_id);
    hipError_t e = bb::launch_math_probe(fn, x, y, out, n, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "launch math probe");
    return BB_OK;
}

// Diagnostic (not in the public header): bbm's short-path divide / square
// root against the IEEE operations on the device (bb_common.hip
// k_divsqrt_probe); counts[blocks] mismatches, ex[2 * blocks] one example each.
int bb_diag_divsqrt(int32_t mode, uint64_t start, uint64_t count, uint32_t seed, uint32_t *counts, uint32_t *ex,
                    int32_t blocks, int32_t gpu_id, void *stream)
{
    if (!counts || !ex || blocks <= 0 || mode < 0 || mode > 5) return fail(BB_ERR_INVALID_ARG, "bb_diag_divsqrt");
    DeviceGuard g(gpu_id);
    hipError_t e = bb::launch_divsqrt_probe(mode, start, count, seed, counts, ex, blocks, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "launch divsqrt probe");
    return BB_OK;
}

// Diagnostic (not in the public header): one k_policy launch over `rows`
// rows with per-wave phase clocks (bb_policy.hip pol_trace) copied to
// out[waves][POL_TRACE_POINTS]; *waves = the launch's waves.
int bb_diag_policy_trace(const bb_policy_weights *w, int32_t gpu_id, const float *obs, int64_t rows,
                         int64_t obs_stride, int32_t stochastic, void *stream, uint64_t *out, int64_t max_waves,
                         int64_t *waves)
{
    if (!weights_ok(w) || !obs || rows <= 0 || !out || !waves) return fail(BB_ERR_INVALID_ARG, "bb_diag_policy_trace");
    DeviceGuard g(gpu_id);
    hipStream_t st = (hipStream_t)stream;
    const int64_t cap = 1 << 16;
    bb::PolicyArgs a{};
    a.w = policy_weights(w);
    a.obs = obs; a.obs_stride = obs_stride; a.rows = rows;
    a.stochastic = stochastic ? 1 : 0; a.seed = 1; a.step = 2;
    if (hipMalloc(&a.diag_ts, (size_t)cap * bb::POL_TRACE_POINTS * 8) != hipSuccess) return fail(BB_ERR_OOM, "trace");
    (void)hipMemsetAsync(a.diag_ts, 0, (size_t)cap * bb::POL_TRACE_POINTS * 8, st);
    hipError_t e = bb::launch_policy(a, st);
    if (e == hipSuccess) e = bb::launch_policy(a, st);
    const int64_t n = max_waves < cap ? max_waves : cap;
    if (e == hipSuccess) e = hipMemcpyAsync(out, a.diag_ts, (size_t)n * bb::POL_TRACE_POINTS * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(a.diag_ts);
    if (e != hipSuccess) return hip_fail(e, "policy trace");
    *waves = n;
    return BB_OK;
}

int64_t bb_algorithmic_bytes_per_world(int32_t n)
{
    // B(N) = N (268 + 4 obs_used(N)) + 152
    return (int64_t)n * (268 + 4 * (int64_t)bb::obs_used(n)) + 152;
}

int32_t bb_rollout_fused(int32_t n) { return bb::fused_rollout_n(n) ? 1 : 0; }

int64_t bb_rollout_bytes_per_world_step(int32_t n)
{
    // per step and agent: action row in (24 B), observation row (4 obs_used),
    // reward and done (8 B) out
    return (int64_t)n * (32 + 4 * (int64_t)bb::obs_used(n));
}

int64_t bb_rollout_state_bytes_per_world(int32_t n)
{
    // once per launch: the B(N) state columns except the per-step action read
    // and observation write (loaded at the start, stored after the last step)
    return bb_algorithmic_bytes_per_world(n) - (int64_t)n * (24 + 4 * (int64_t)bb::obs_used(n));
}

int32_t bb_rollout_policy_path(const bb_sim *s, int32_t with_opponent, uint32_t flags)
{
    if (!s) return fail(BB_ERR_INVALID_ARG, "bb_rollout_policy_path: sim");
    const int32_t path = ppo_path(s, with_opponent != 0, flags);
    if (path < 0) return fail(BB_ERR_UNSUPPORTED, "bb_rollout_policy_path: the reference's 2-agent game only");
    return path;
}

int64_t bb_rollout_policy_bytes(const bb_sim *s, int32_t with_opponent, uint32_t flags, int32_t n)
{
    if (!s || n < 1) return 0;
    if (s->n != 2) return fail(BB_ERR_UNSUPPORTED, "bb_rollout_policy_bytes: the reference's 2-agent game only");
    const int64_t B = bb_algorithmic_bytes_per_world(2);
    const int64_t row = 4 * (int64_t)bb::obs_used(2);   // a sim observation row's values (412 B)
    const int64_t rec = 4 * (int64_t)bb::POL_IN;        // a buffer.obs row (128 floats)
    const int64_t outs = 24 + 4 + 4;                    // buffer.actions, log_probs, values
    const int64_t rd = 4 + 4;                           // buffer.rewards, not_dones
    // the first policy pass: the trainee's sim row in, buffer.obs[0], the
    // action row into the sim, the outputs; the value pass: next_value
    const int64_t pass0 = rec + rec + 24 + outs;
    switch (ppo_path(s, with_opponent != 0, flags)) {
    case BB_PPO_PATH_FUSED_ROLLOUT:
        // state in once and out once (every row of the last step included); per
        // step the policy's records and the step's reward / done
        return B + (int64_t)n * (rec + outs + rd) + 4;
    case BB_PPO_PATH_FUSED_STEP:
        // what the call must move, not what the launch does: the state in once
        // and out once (B, the last step's rows included), the trainee's rows
        // read by the first policy pass, per step the records, the value pass's
        // next_value.  (k_rollout_ppo also round-trips each step's state and
        // action rows through memory -- L2 hits mostly, its PMC traffic is
        // 2x these bytes -- which the fused rollout's registers avoid.)
        return B + rec + (int64_t)n * (rec + outs + rd) + 4;
    default:
        // per step: the world step (the trainee's row into buffer.obs[k+1]
        // instead of the sim from step 0 to n-2), then a policy pass reading
        // that row back, the outputs, the reward / done read from the sim and
        // recorded; then the value pass reads the last rows
        return pass0 + (int64_t)(n - 1) * (B - row + rec + rec + 24 + outs + rd + rd) + B + rd + rd + rec + 4;
    }
}

const char *bb_last_error(void) { return g_err.c_str(); }

}  // extern "C"
