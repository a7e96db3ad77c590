// bb_sim.h -- the basketball world step, compiled for gfx950 and for the host.
//
// One world = one register-resident `World<N>`; `step_world` runs the 19
// systems of the reference task graph (src/game.cpp:1463-1526) in graph order,
// agents in creation order, exactly as the Madrona CPU TaskGraphExecutor
// sequences them.  The gfx950 kernel (bb_step.hip) maps one world to one lane:
// load -> step_world -> store, so every cross-entity `ctx.get<>` of the
// reference becomes a register access.
//
// HBM layout = the reference's export layout (world-major component columns,
// src/mgr.cpp:317-445) for every exported component, plus world-major columns
// for the build-internal state (velocity, cooldown, ...).  See DESIGN.md.
#pragma once
#include <stdint.h>
#include <type_traits>
#include "bb_math.h"
#include "bb_rng.h"

namespace bb {

// ------------------------------------------------------------------ constants
// src/constants.hpp, evaluated in float exactly like the C++ constexprs.
constexpr float PI = 3.14159265358979323846f;                 // madrona::math::pi
constexpr float TS = 1.0f / 62.0f;                            // :12
constexpr float TIME_PER_PERIOD = 10.f;                       // :13
constexpr float PPM = 110.f;                                  // :17
constexpr float HOOP_ZONE = 0.1f;                             // :24
constexpr float AGENT_SIZE = 0.2f;                            // :39
constexpr float SHOULDER = 0.4290;                            // :40
constexpr float DEPTH = .1;                                   // :41
constexpr float GUARD = .2f;                                  // :45
constexpr float START_STD = 5.f;                              // :46
constexpr float DEFAULT_SPEED = 3.f;                          // :47
constexpr float DEF_SLOW = 0.2f;                              // :48
constexpr float DEF_REACT = 10.f;                             // :49
constexpr float SPAWN_R = 8.f;                                // :50
constexpr float ANGLE_STEP = PI / 4.0f;                       // :53
constexpr float BALL_SLOW = 0.9f;                             // :55
constexpr float DIST_DEV = .008f, DEF_DEV = .002f, VEL_DEV = .001f;  // :59-61
constexpr float COURT_L = 28.65f, COURT_W = 15.24f;          // :67-68
constexpr float WORLD_W = COURT_L * 1.1f;                     // :72
constexpr float WORLD_H = COURT_W * 1.1f;                     // :73
constexpr float CMINX = (WORLD_W - COURT_L) / 2.0f;           // :76
constexpr float CMAXX = CMINX + COURT_L;                      // :77
constexpr float CMINY = (WORLD_H - COURT_W) / 2.0f;           // :78
constexpr float CMAXY = CMINY + COURT_W;                      // :79
constexpr float HOOP_FROM_BASE = 1.575f;                      // :84
constexpr float ARC = 7.24f, CORNER_SIDE = 0.91f, CORNER_LEN = 4.27f;  // :91-93
constexpr float CORNER_LO_Y = CMINY + CORNER_SIDE;            // helper.cpp:55
constexpr float CORNER_HI_Y = CMINY + COURT_W - CORNER_SIDE;  // helper.cpp:56
constexpr float CORNER_LEFT_X = CMINX + CORNER_LEN;           // helper.cpp:63
constexpr float CORNER_RIGHT_X = CMINX + COURT_L - CORNER_LEN;  // helper.cpp:67
constexpr float HALF_WORLD_W = WORLD_W / 2.0f;                // helper.cpp:60
constexpr float INBOUND_DY = PPM / 60;                        // game.cpp:918
constexpr float HALF_SHOULDER = SHOULDER / 2.0f;              // game.cpp:561
constexpr float HALF_DEPTH = DEPTH / 2.0f;                    // game.cpp:562
constexpr float TURN_POS = (PI / 180.f) * 6;                  // game.cpp:423
constexpr float TURN_NEG = (PI / 180.f) * -6;
constexpr float PI_OVER_8 = PI / 8.f;                         // game.cpp:747
constexpr int32_t PH = 2147483647;                            // ENTITY_ID_PLACEHOLDER
// Build-defined entity ids (creation order of src/gen.cpp:101-206).
constexpr int32_t HOOP0_ID = 0, HOOP1_ID = 1, BALL_ID = 2, AGENT0_ID = 3;

constexpr uint32_t FLAG_PER_WORLD_RNG = 0x1u, FLAG_NO_TAG_MASK = 0x2u, FLAG_FULL_GAME = 0x4u;

BB_HD constexpr int obs_used(int n) { return 61 + 38 * (n - 1) + 2 * n; }
// BB_OBS_ROW_ALIGN (floats, diagnostic builds): rows wider than 128 floats
// (N > 2) end on this boundary; the product keeps 4 (16-byte pieces).
#ifndef BB_OBS_ROW_ALIGN
#define BB_OBS_ROW_ALIGN 4
#endif
BB_HD constexpr int obs_width(int n)
{
    return ((obs_used(n) + 3) & ~3) < 128
               ? 128
               : ((obs_used(n) + BB_OBS_ROW_ALIGN - 1) / BB_OBS_ROW_ALIGN * BB_OBS_ROW_ALIGN);
}

// ------------------------------------------------------------------ vec math
// madrona::math::Vector3 / Quat operations, in the reference's operand order.
struct F3 { float x, y, z; };
struct Q4 { float w, x, y, z; };
BB_HD F3 f3(float x, float y, float z) { F3 r; r.x = x; r.y = y; r.z = z; return r; }
BB_HD F3 operator+(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
BB_HD F3 operator-(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
BB_HD F3 operator-(F3 a) { return f3(-a.x, -a.y, -a.z); }
BB_HD F3 operator*(F3 a, float s) { return f3(a.x * s, a.y * s, a.z * s); }
BB_HD float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
BB_HD float len2(F3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
BB_HD float len(F3 a) { return bbm::sqrtf_(len2(a)); }
// Vector3::normalize: unpinned Madrona detail, fixed as v * (1 / |v|).
BB_HD F3 norm(F3 a) { return a * (1.0f / bbm::sqrtf_(len2(a))); }
BB_HD F3 cross(F3 a, F3 b)
{
    return f3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
BB_HD float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
BB_HD float minf(float a, float b) { return b < a ? b : a; }
BB_HD float maxf(float a, float b) { return b > a ? b : a; }
BB_HD Q4 quat_axis_z(float angle, float axis_z)  // Quat::angleAxis(angle, {0,0,axis_z})
{
    float s, c;
    bbm::sincosf_(0.5f * angle, &s, &c);
    Q4 q; q.w = c; q.x = s * 0.f; q.y = s * 0.f; q.z = s * axis_z; return q;
}
BB_HD Q4 quat_axis(float angle, F3 n)
{
    float s, c;
    bbm::sincosf_(0.5f * angle, &s, &c);
    Q4 q; q.w = c; q.x = s * n.x; q.y = s * n.y; q.z = s * n.z; return q;
}
BB_HD Q4 qmul(Q4 a, Q4 b)
{
    Q4 r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x;
    r.z = a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w;
    return r;
}
// Quat::rotateVec (pinned by scripts/viewer.py:59-65)
BB_HD F3 rotate(Q4 q, F3 v)
{
    const F3 p = f3(q.x, q.y, q.z);
    const F3 pv = cross(p, v);
    const F3 ppv = cross(p, pv);
    return v + ((pv * q.w) + ppv) * 2.f;
}
// rotate(q, (0,1,0)), the agent's forward vector
BB_HD F3 forward(Q4 q) { return rotate(q, f3(0.f, 1.f, 0.f)); }

// findRotationBetweenVectors(AGENT_BASE_FORWARD, t)  (src/helper.cpp:14-42)
BB_HD Q4 rotation_from_forward(F3 t)
{
    const F3 a = norm(f3(0.f, 1.f, 0.f));
    t = norm(t);
    const float d = dot(a, t);
    if (d > 0.999999f) { Q4 id; id.w = 1.f; id.x = 0.f; id.y = 0.f; id.z = 0.f; return id; }
    if (d < -0.999999f) return quat_axis_z(PI, 1.f);
    const F3 ax = norm(cross(a, t));
    return quat_axis(bbm::acosf_(d), ax);
}

// getShotPointValue (src/helper.cpp:50-81); arc_ge2: Params::arc_ge2 (the
// distance test d >= ARC on the squared distance, no root)
BB_HD int32_t shot_point_value(F3 p, F3 hz, float arc_ge2)
{
    const float d2 = len2(p - hz);
    if (p.y < CORNER_LO_Y || p.y > CORNER_HI_Y) {
        if (hz.x < HALF_WORLD_W) { if (p.x <= CORNER_LEFT_X) return 3; }
        else { if (p.x >= CORNER_RIGHT_X) return 3; }
    }
    return d2 >= arc_ge2 ? 3 : 2;
}

// c ? a : b, word by word for aggregates (a ?: on structs selects between
// their addresses, which leaves the operands in scratch memory).
template <class T>
BB_HD T sel(bool c, const T &a, const T &b)
{
    if constexpr (std::is_arithmetic<T>::value) {
        return c ? a : b;
    } else {
        static_assert(sizeof(T) % 4 == 0, "32-bit words");
        constexpr int NW = sizeof(T) / 4;
        uint32_t x[NW], y[NW];
        __builtin_memcpy(x, &a, sizeof(T));
        __builtin_memcpy(y, &b, sizeof(T));
#pragma unroll
        for (int q = 0; q < NW; q++) x[q] = c ? x[q] : y[q];
        T r;
        __builtin_memcpy(&r, x, sizeof(T));
        return r;
    }
}

// A kernel-argument value read as a wave-uniform scalar: a runtime choice
// between two of them stays a register select instead of becoming a per-lane
// load from the argument segment (select-of-loads -> load-of-select).
BB_HD float uni(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, x)));
#else
    return x;
#endif
}
BB_HD F3 uni(F3 a) { return f3(uni(a.x), uni(a.y), uni(a.z)); }
// A kernel-argument value used as it is: uni() without the readfirstlane.
// The identity itself hides nothing from the optimiser; what changes the
// generated code is the missing readfirstlane, which is convergent and keeps
// every branch around it from being if-converted (the values are uniform
// kernel arguments, held in scalar registers anyway).
BB_HD float sconst(float x)
{
    return x;
}
BB_HD F3 sconst(F3 a) { return f3(sconst(a.x), sconst(a.y), sconst(a.z)); }
BB_HD Q4 uni(Q4 q)
{
    Q4 r;
    r.w = uni(q.w); r.x = uni(q.x); r.y = uni(q.y); r.z = uni(q.z);
    return r;
}
BB_HD Q4 sconst(Q4 q)
{
    Q4 r;
    r.w = sconst(q.w); r.x = sconst(q.x); r.y = sconst(q.y); r.z = sconst(q.z);
    return r;
}

// Agent held by slot `slot` of agent k's view: k itself, then the other
// agents in creation order.
template <int N>
BB_HD constexpr int view_source(int slot, int k)
{
    return slot == 0 ? k : ((slot - 1) < k ? slot - 1 : slot);
}

// Slot of agent i in agent k's view (the inverse of view_source).
template <int N>
BB_HD constexpr int view_slot(int i, int k)
{
    return i == k ? 0 : (i < k ? i + 1 : i);
}

// From this agent count on the GPU kernel keeps the world in LDS
// (bb_kernels.hip, Lanes::SHARED), where an indexed access is one LDS load.
#ifndef BB_LDS_WORLD_MIN_N
#define BB_LDS_WORLD_MIN_N 4
#endif
constexpr int LDS_WORLD_MIN_N = BB_LDS_WORLD_MIN_N;

// Value of f(j) for j == i.  For register-resident worlds (N < 4) it is built
// from selects: i may be a runtime value -- e.g. the lane's agent -- while
// every array index inside f stays constant, so nothing goes to scratch.  For
// worlds in LDS (and on the host) f(i) indexes directly.
template <int N, class F>
BB_HD auto pick_by(int i, F f) -> decltype(f(0))
{
    if constexpr (N >= LDS_WORLD_MIN_N) {
        return f(i);
    } else {
        auto r = f(0);
#pragma unroll
        for (int j = 1; j < N; j++) r = sel(i == j, f(j), r);
        return r;
    }
}

// How per-agent work is spread over lanes.  EachAgent: the calling lane
// computes every agent's result (host executor, one lane per world).  The
// agent-lane kernel (bb_kernels.hip) passes a policy that computes only the
// lane's own agent and collects the others from the neighbouring lanes of
// the same world.  f(i) may read anything but must not write the world.
// mark(point): timing hook between groups of systems (no-op here; the
// kernel's trace variant records a clock).
struct EachAgent {
    template <class T, int N, class F>
    BB_HD void all(F f, T (&out)[N]) const
    {
#pragma unroll
        for (int i = 0; i < N; i++) out[i] = f(i);
    }
    // Per-agent system whose agent i reads nothing another agent's apply
    // writes: every f(i) from the state before the system, then apply(i, .)
    // in creation order.  (A kernel whose lanes share the world in LDS lets
    // each lane apply only its own agent's result, see bb_kernels.hip.)
    template <int N, class F, class P>
    BB_HD void each(F f, P apply) const
    {
        decltype(f(0)) out[N];
        all(f, out);
#pragma unroll
        for (int i = 0; i < N; i++) apply(i, out[i]);
    }
    BB_HD void mark(int) const {}
};

// ------------------------------------------------------------------ layout
// Column pointers.  Exported columns keep the reference byte layouts;
// *_u views reinterpret mixed int/float structs (GameState, Team, Stats).
struct Columns {
    int32_t *reset;        // [W][N]            Reset
    uint32_t *game_state;  // [W][14]           GameState (mixed i32/f32, exported as f32)
    int32_t *action;       // [W][N][6]         Action
    int32_t *action_mask;  // [W][N][4]         ActionMask
    float *agent_pos;      // [W][N][3]         Position
    float *obs;            // [W][N][OBSW]      Observations
    float *reward;         // [W][N]            Reward
    float *done;           // [W][N]            Done
    int32_t *agent_id;     // [W][N]            Entity (build ids)
    int32_t *possession;   // [W][N][3]         InPossession
    float *orientation;    // [W][N][4]         Orientation (w,x,y,z)
    uint32_t *team;        // [W][N][5]         Team {i32, f32 x3, i32}
    float *stats;          // [W][N][2]         Stats (exported as i32)
    float *ball_pos;       // [W][1][3]
    int32_t *ball_physics; // [W][1][7]
    int32_t *ball_id;      // [W][1]
    int32_t *ball_grabbed; // [W][1][2]
    float *ball_vel;       // [W][1][3]
    float *hoop_pos;       // [W][2][3]
    // build-internal state
    float *agent_vel;      // [W][N][3]
    float *cooldown;       // [W][N]
    uint32_t *cur_step;    // [W][N]
    int32_t *inbounding;   // [W][N][2]
    float *attributes;     // [W][N][10]  maxSpeed quick shoot ft react tgt.xyz shotPct pad
    int32_t *world_clock;  // [W]
    uint32_t *rng_counter; // [W]
};

struct Params {
    Columns c;
    int64_t num_worlds;
    int64_t world_offset;
    float width, height, start_x, start_y;
    float hoop0[3], hoop1[3];
    uint32_t seed, flags;
    // Derived tables, computed once on the host with the very functions the
    // step would call (so a table hit is bit-identical to the evaluation):
    float mv_sin[8], mv_cos[8];  // sincos((float)k * pi/4), k = moveAngle in [0, 8)
    Q4 turn_q[2];                // angleAxis(+6 deg, z), angleAxis(-6 deg, z)   game.cpp:423-424
    Q4 start_q[2];               // angleAxis(-pi/2, z), angleAxis(+pi/2, z)     gen.cpp:196
    float rot_thresh;            // (float)acos(c) > pi/8  <=>  c < rot_thresh   game.cpp:746-747
    int32_t rot_exact;           // 1: threshold not verified, evaluate acos
    // sqrtf is correctly rounded, hence monotone: sqrtf(t) <= c  <=>  t <= T
    // with T the largest such float, and sqrtf(t) < c  <=>  t < T' with T'
    // the smallest float whose root is >= c.  Distance tests against
    // constants compare squared lengths with these (no root taken).
    float grab_le2;              // len <= 0.3                                  game.cpp:202
    float touch_le2;             // len <= AGENT_SIZE                           game.cpp:1045
    float hoop_le2;              // sqrt(dx^2 + dy^2) <= HOOP_SCORE_ZONE_SIZE   game.cpp:885-888
    float near_lt2;              // len < 2 (the shot's defender deviation)    game.cpp:329
    float arc_ge2;               // len >= THREE_POINT_RADIUS                  helper.cpp:80
    uint32_t diag_skip;          // diagnostics only (MODE_SKIP): systems to leave out
    uint32_t diag_dup;           // diagnostics only (MODE_SKIP): systems to run twice
    uint32_t diag_keep;          // diagnostics only: 0 (the duplicate run's result is dropped)
    uint64_t *diag_ts;           // diagnostics only (MODE_TRACE): TRACE_POINTS clocks per wave
    // PPO's buffer.obs record (bb_rollout_policy, scripts/ppo.py:129; N = 2):
    // when set, the step also writes agent rec_agent's observation row of
    // world w to rec_obs + w * 128 (the whole 128 floats, zero tail included)
    float *rec_obs;
    int32_t rec_agent;
    // with rec_obs: agent rec_agent's row goes to rec_obs only, not to the
    // sim's obs (PPO's per-step loop reads it there; the last step of the
    // rollout writes every row as usual)
    int32_t rec_only;
};

BB_HD uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
BB_HD float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }

// Vector-width chunk load/store of NW consecutive 32-bit words (16-B, 8-B or
// 4-B wide accesses depending on the chunk's alignment).
template <int NW>
BB_HD void load_words(const void *base, int64_t w, uint32_t (&o)[NW])
{
    const uint32_t *p = (const uint32_t *)base + w * NW;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (NW % 4 == 0) {
#pragma unroll
        for (int k = 0; k < NW / 4; k++) {
            const uint4 v = ((const uint4 *)p)[k];
            o[4 * k] = v.x; o[4 * k + 1] = v.y; o[4 * k + 2] = v.z; o[4 * k + 3] = v.w;
        }
    } else if constexpr (NW % 2 == 0) {
#pragma unroll
        for (int k = 0; k < NW / 2; k++) {
            const uint2 v = ((const uint2 *)p)[k];
            o[2 * k] = v.x; o[2 * k + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < NW; k++) o[k] = p[k];
    }
#else
    __builtin_memcpy(o, p, sizeof(o));
#endif
}

// AUX: cache-policy bits of the device stores (-1: plain global stores;
// otherwise buffer stores with these aux bits -- gfx950: 2 nt, 16 sc1; `base`
// must then be wave-uniform, the column's own base).
template <int NW, int AUX = -1>
BB_HD void store_words(void *base, int64_t w, const uint32_t (&o)[NW])
{
    uint32_t *p = (uint32_t *)base + w * NW;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (AUX >= 0) {
        // Wave-uniform descriptor 63 chunks below the first active lane's
        // chunk: a lane's offset (w - wf + 63 chunks) is >= 0 for any lane
        // whose chunk lies at most 63 chunks before the first active lane's
        // -- every caller's lanes store chunks of the wave's own <= 64 rows,
        // in whatever lane order -- and stays small at any column size.
        // (Only the descriptor's base address may lie before the column; no
        // access does.)
        const uint64_t wu = (uint64_t)w;
        const int64_t wf = (int64_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(wu >> 32)) << 32) |
                                     __builtin_amdgcn_readfirstlane((uint32_t)wu)) - 63;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc((uint32_t *)base + wf * NW, 0, 0x7fffffff, 0x00020000);
        const int off = (int)((w - wf) * NW * 4);
        typedef uint32_t u2 __attribute__((ext_vector_type(2)));
        typedef uint32_t u3 __attribute__((ext_vector_type(3)));
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        if constexpr (NW % 4 == 0) {
#pragma unroll
            for (int k = 0; k < NW / 4; k++)
                __builtin_amdgcn_raw_buffer_store_b128(u4{o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]}, rs,
                                                       off + 16 * k, 0, AUX);
        } else if constexpr (NW % 2 == 0) {
#pragma unroll
            for (int k = 0; k < NW / 2; k++)
                __builtin_amdgcn_raw_buffer_store_b64(u2{o[2 * k], o[2 * k + 1]}, rs, off + 8 * k, 0, AUX);
        } else if constexpr (NW == 3) {
            __builtin_amdgcn_raw_buffer_store_b96(u3{o[0], o[1], o[2]}, rs, off, 0, AUX);
        } else {
#pragma unroll
            for (int k = 0; k < NW; k++) __builtin_amdgcn_raw_buffer_store_b32(o[k], rs, off + 4 * k, 0, AUX);
        }
        return;
    }
    if constexpr (NW % 4 == 0) {
#pragma unroll
        for (int k = 0; k < NW / 4; k++)
            ((uint4 *)p)[k] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
    } else if constexpr (NW % 2 == 0) {
#pragma unroll
        for (int k = 0; k < NW / 2; k++) ((uint2 *)p)[k] = make_uint2(o[2 * k], o[2 * k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < NW; k++) p[k] = o[k];
    }
#else
    __builtin_memcpy(p, o, sizeof(o));
#endif
}

BB_HD void store_f4(float *p, float a, float b, float c, float d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    *(float4 *)p = make_float4(a, b, c, d);
#else
    p[0] = a; p[1] = b; p[2] = c; p[3] = d;
#endif
}

// Fill the derived tables of Params (host).  Every entry is produced by the
// same deterministic function the step would evaluate.
inline bool rot_pred(float c) { return (float)bbm::acos_d((double)c) > PI_OVER_8; }

// T(c) = the largest float t in [0, inf) with sqrtf(t) <= c; T'(c) = the
// smallest with sqrtf(t) >= c (bisection over bit patterns: sqrtf is monotone)
inline float sqrt_le_bound(float c)
{
    uint32_t lo = 0, hi = fbits(__builtin_inff());  // sqrtf(lo) <= c, sqrtf(hi) > c
    while (hi - lo > 1u) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (bbm::sqrtf_(bitsf(mid)) <= c) lo = mid; else hi = mid;
    }
    return bitsf(lo);
}
inline float sqrt_ge_bound(float c)
{
    uint32_t lo = 0, hi = fbits(__builtin_inff());  // sqrtf(lo) < c, sqrtf(hi) >= c
    while (hi - lo > 1u) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (bbm::sqrtf_(bitsf(mid)) < c) lo = mid; else hi = mid;
    }
    return bitsf(hi);
}

inline void build_tables(Params &p)
{
    p.grab_le2 = sqrt_le_bound(0.3f);
    p.touch_le2 = sqrt_le_bound(AGENT_SIZE);
    p.hoop_le2 = sqrt_le_bound(HOOP_ZONE);
    p.near_lt2 = sqrt_ge_bound(2.0f);
    p.arc_ge2 = sqrt_ge_bound(ARC);
    for (int k = 0; k < 8; k++) bbm::sincosf_((float)k * ANGLE_STEP, &p.mv_sin[k], &p.mv_cos[k]);
    p.turn_q[0] = quat_axis_z(TURN_POS, 1.f);
    p.turn_q[1] = quat_axis_z(TURN_NEG, 1.f);
    p.start_q[0] = quat_axis_z(-PI / 2.0f, 1.f);  // == start_orientation_eval(0)
    p.start_q[1] = quat_axis_z(PI / 2.0f, 1.f);   // == start_orientation_eval(1)
    // bisection over float bit patterns in [0.5, 1]: pred(lo) true, pred(hi) false
    uint32_t lo = fbits(0.5f), hi = fbits(1.0f);
    if (!rot_pred(bitsf(lo)) || rot_pred(bitsf(hi))) { p.rot_exact = 1; p.rot_thresh = 0.f; return; }
    while (hi - lo > 1u) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (rot_pred(bitsf(mid))) lo = mid; else hi = mid;
    }
    p.rot_thresh = bitsf(hi);
    p.rot_exact = 0;
    // verify c < T  <=>  pred(c) on a window of 2^17 floats around T
    for (int64_t k = -65536; k <= 65536; k++) {
        const float cval = bitsf((uint32_t)((int64_t)hi + k));
        if (rot_pred(cval) != (cval < p.rot_thresh)) { p.rot_exact = 1; return; }
    }
}

// ------------------------------------------------------------------ state
template <int N>
struct World {
    // GameState singleton (src/types.hpp:46-67)
    int32_t g_inb, g_live; float g_period, g_poss; int32_t g_h0; float g_s0; int32_t g_h1;
    float g_s1, g_clock, g_shot, g_bask, g_oob, g_inbclk; int32_t g_1v1;
    int32_t reset_now;   // WorldClock singleton
    uint32_t rng_ctr;    // Sim::rng draw counter
    // agents
    int32_t rst[N], act[N][6], msk[N][4];
    float cd[N], px[N], py[N], pz[N], rew[N], done[N];
    uint32_t step[N];
    int32_t has[N], bid[N], pw[N];
    float qw[N], qx[N], qy[N], qz[N];
    int32_t inb[N], allow[N], team[N], dhoop[N];
    float attr[N][10];   // maxSpeed quickness shooting ft reaction tx ty tz shotPct pad
    float vx[N], vy[N], vz[N];
    // ball
    float bx, by, bz, bvx, bvy, bvz;
    int32_t fl, lta, ltt, sba, sbt, spv, gin;  // BallPhysics
    int32_t grab, holder;                      // Grabbed

    BB_HD F3 pos(int i) const { return f3(px[i], py[i], pz[i]); }
    BB_HD void set_pos(int i, F3 v) { px[i] = v.x; py[i] = v.y; pz[i] = v.z; }
    BB_HD F3 vel(int i) const { return f3(vx[i], vy[i], vz[i]); }
    BB_HD void set_vel(int i, F3 v) { vx[i] = v.x; vy[i] = v.y; vz[i] = v.z; }
    BB_HD Q4 q(int i) const { Q4 r; r.w = qw[i]; r.x = qx[i]; r.y = qy[i]; r.z = qz[i]; return r; }
    BB_HD void set_q(int i, Q4 v) { qw[i] = v.w; qx[i] = v.x; qy[i] = v.y; qz[i] = v.z; }
    BB_HD F3 bpos() const { return f3(bx, by, bz); }
    BB_HD void set_bpos(F3 v) { bx = v.x; by = v.y; bz = v.z; }
    BB_HD F3 bvel() const { return f3(bvx, bvy, bvz); }
    BB_HD void set_bvel(F3 v) { bvx = v.x; bvy = v.y; bvz = v.z; }
    BB_HD F3 target(int i) const { return f3(attr[i][5], attr[i][6], attr[i][7]); }
    BB_HD void set_target(int i, F3 v) { attr[i][5] = v.x; attr[i][6] = v.y; attr[i][7] = v.z; }
};

// Per-world execution context: world index, RNG key cache, side channel for
// the rarely written columns (Stats, Team colour) that are not kept in
// registers.
struct Ctx {
    const Params *p;
    int64_t w;
    bool writer;   // this lane performs the world's memory side effects
    const double *erf_tab;  // bbm::ERF_TAYLOR (the GPU kernels: its copy in LDS)
};

BB_HD Ctx make_ctx(const Params &p, int64_t w, bool writer = true)
{
    Ctx c; c.p = &p; c.w = w; c.writer = writer; c.erf_tab = &bbm::ERF_TAYLOR[0][0]; return c;
}

// sampleUniform at stream position ctr of the world's stream
template <int N>
BB_HD float sample_uniform_at(const World<N> &s, const Ctx &c, uint32_t ctr, float lo, float hi)
{
    const uint32_t k = (c.p->flags & FLAG_PER_WORLD_RNG) ? (uint32_t)(c.p->world_offset + c.w) : 0u;
    uint32_t r0, r1;
    threefry2x32(c.p->seed, k, ctr, 0u, &r0, &r1);
    return lo + (hi - lo) * u01_from_bits(r0);
}

template <int N>
BB_HD float sample_uniform(World<N> &s, Ctx &c, float lo, float hi)
{
    // world key {seed, k}: k = 0 for every world (reference: one shared key,
    // src/sim.cpp:89) or the global world index (per-world streams)
    const uint32_t k = (c.p->flags & FLAG_PER_WORLD_RNG) ? (uint32_t)(c.p->world_offset + c.w) : 0u;
    uint32_t r0, r1;
    threefry2x32(c.p->seed, k, s.rng_ctr, 0u, &r0, &r1);
    s.rng_ctr++;
    return lo + (hi - lo) * u01_from_bits(r0);
}

template <int N>
BB_HD F3 hoop_pos(const Ctx &c, int h)
{
    const F3 h0 = sconst(f3(c.p->hoop0[0], c.p->hoop0[1], c.p->hoop0[2]));
    const F3 h1 = sconst(f3(c.p->hoop1[0], c.p->hoop1[1], c.p->hoop1[2]));
    return sel(h == 0, h0, h1);
}

BB_HD F3 vec_to_center(const Ctx &c, F3 p)  // findVectorToCenter, helper.cpp:44-48
{
    return norm(f3(c.p->start_x, c.p->start_y, 0.f) - p);
}

// ------------------------------------------------------------------ gen/reset
BB_HD Q4 start_orientation_eval(int i)  // gen.cpp:196 / :277
{
    return (i % 2 == 0) ? quat_axis_z(-PI / 2.0f, 1.f) : quat_axis_z(PI / 2.0f, 1.f);
}

template <int N>
BB_HD Q4 start_orientation(const Ctx &c, int i)
{
    return sel(i % 2 == 0, sconst(c.p->start_q[0]), sconst(c.p->start_q[1]));
}

// setupAgentPositions (src/helper.cpp:108-160); returns the ball holder id.
template <int N>
BB_HD int32_t setup_agent_positions(World<N> &s, Ctx &c, F3 *ball_at)
{
    int32_t off_id = PH;
#pragma unroll
    for (int i = 0; i < N; i++) {
        if (s.g_1v1 == 1) {
            if (i == 0) {
                const F3 base = f3(c.p->start_x + ((float)i * 2.f), c.p->start_y, 0.f);
                const float xd = sample_uniform(s, c, -START_STD, START_STD);
                const float yd = sample_uniform(s, c, -START_STD, START_STD);
                F3 p = base + f3(xd, yd, 0.f);
                p.x = clampf(p.x, 0.f, c.p->width);
                p.y = clampf(p.y, 0.f, c.p->height);
                s.set_pos(i, p);
                *ball_at = p;
                off_id = AGENT0_ID + i;
                s.has[i] = 1; s.bid[i] = BALL_ID; s.pw[i] = 2;
            } else {
                const float ang = sample_uniform(s, c, 0.f, 2.f * PI);
                float sn, cs;
                bbm::sincosf_(ang, &sn, &cs);
                F3 p = *ball_at + f3(SPAWN_R * cs, SPAWN_R * sn, 0.f);
                p.x = clampf(p.x, 0.f, c.p->width);
                p.y = clampf(p.y, 0.f, c.p->height);
                s.set_pos(i, p);
                s.has[i] = 0; s.bid[i] = PH; s.pw[i] = 2;
            }
        } else {
            s.set_pos(i, f3((c.p->start_x - 1.f) - (float)(-2 * (i % 2)),
                            (c.p->start_y - 2.f) + (float)(i / 2), 0.f));
            if (i == 0) { off_id = AGENT0_ID + i; s.has[i] = 1; s.bid[i] = BALL_ID; s.pw[i] = 2; }
            else { s.has[i] = 0; s.bid[i] = PH; s.pw[i] = 2; }
        }
        s.attr[i][0] = DEFAULT_SPEED - (float)i * DEF_SLOW;
        s.attr[i][1] = 1.f; s.attr[i][2] = 0.f; s.attr[i][3] = 0.f;
        s.attr[i][4] = (float)i * DEF_REACT;
        s.set_target(i, s.pos(i));
        s.attr[i][8] = 0.f; s.attr[i][9] = 0.f;
    }
    return off_id;
}

// Team column write (rare: generation and resets).
template <int N>
BB_HD void write_team(const Ctx &c, int i, int32_t team, F3 color, int32_t dhoop)
{
    uint32_t *t = c.p->c.team + (c.w * N + i) * 5;
    t[0] = (uint32_t)team; t[1] = fbits(color.x); t[2] = fbits(color.y); t[3] = fbits(color.z);
    t[4] = (uint32_t)dhoop;
}

// generateWorld (src/gen.cpp:13-214) + Sim::Sim rng seeding (src/sim.cpp:86-96)
template <int N>
BB_HD void generate_world(World<N> &s, Ctx &c)
{
    s.g_inb = 0; s.g_live = 1; s.g_period = 1.f; s.g_poss = 0.f; s.g_h0 = HOOP0_ID; s.g_s0 = 0.f;
    s.g_h1 = HOOP1_ID; s.g_s1 = 0.f; s.g_clock = TIME_PER_PERIOD; s.g_shot = 24.f; s.g_bask = 0.f;
    s.g_oob = 0.f; s.g_inbclk = 0.f; s.g_1v1 = (c.p->flags & FLAG_FULL_GAME) ? 0 : 1;
    s.reset_now = 0;
    s.rng_ctr = 0;
    s.bx = c.p->start_x; s.by = c.p->start_y; s.bz = 0.f;
    s.grab = 0; s.holder = PH;
    s.fl = 0; s.lta = PH; s.ltt = PH; s.sba = PH; s.sbt = PH; s.spv = 2; s.gin = 0;
    s.bvx = 0.f; s.bvy = 0.f; s.bvz = 0.f;
#pragma unroll
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int k = 0; k < 6; k++) s.act[i][k] = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) s.msk[i][k] = 0;
        s.rst[i] = 0; s.inb[i] = 0; s.allow[i] = 1; s.rew[i] = 0.f; s.done[i] = 0.f; s.step[i] = 0;
        s.set_q(i, start_orientation<N>(c, i));
        s.cd[i] = 0.f;
        s.vx[i] = 0.f; s.vy[i] = 0.f; s.vz[i] = 0.f;
        s.team[i] = i % 2;
        s.dhoop[i] = (i % 2 == 0) ? s.g_h0 : s.g_h1;
        s.has[i] = 0; s.bid[i] = 0; s.pw[i] = 0;
        s.px[i] = 0.f; s.py[i] = 0.f; s.pz[i] = 0.f;
        if (c.writer) {
            write_team<N>(c, i, s.team[i], (i % 2 == 0) ? f3(0.f, 100.f, 255.f) : f3(128.f, 0.f, 128.f),
                          s.dhoop[i]);
            float *st = c.p->c.stats + (c.w * N + i) * 2;
            st[0] = 0.f; st[1] = 0.f;
        }
    }
    F3 ball_at = f3(c.p->start_x, c.p->start_y, 0.f);
    const int32_t off_id = setup_agent_positions(s, c, &ball_at);
    if (s.g_1v1 == 1) { s.grab = 1; s.holder = off_id; }
}

// resetWorld (src/gen.cpp:216-316)
template <int N>
BB_HD void reset_world(World<N> &s, Ctx &c)
{
    if (s.g_clock <= 0.f && (float)s.g_1v1 == 0.f) {
        if (s.g_period < 4.f || s.g_s0 == s.g_s1) {
            s.g_period += 1.f; s.g_clock = TIME_PER_PERIOD; s.g_shot = 24.f; s.g_live = 1; s.g_inb = 0;
        } else {
            s.g_live = 0;
        }
    } else {
        s.g_inb = 0; s.g_live = 1; s.g_period = 1.f; s.g_poss = 0.f; s.g_s0 = 0.f; s.g_s1 = 0.f;
        s.g_clock = TIME_PER_PERIOD; s.g_shot = 24.f; s.g_bask = 0.f; s.g_oob = 0.f; s.g_inbclk = 0.f;
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int k = 0; k < 6; k++) s.act[i][k] = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) s.msk[i][k] = 0;
        s.rst[i] = 0; s.inb[i] = 0; s.allow[i] = 1; s.done[i] = 1.f; s.step[i] = 0;
        s.set_q(i, start_orientation<N>(c, i));
        s.cd[i] = 0.f;
        s.vx[i] = 0.f; s.vy[i] = 0.f; s.vz[i] = 0.f;
        s.team[i] = i % 2;
        s.dhoop[i] = (i % 2 == 0) ? s.g_h0 : s.g_h1;
        if (c.writer) {
            write_team<N>(c, i, s.team[i], (i % 2 == 0) ? f3(0.f, 100.f, 255.f) : f3(255.f, 0.f, 100.f),
                          s.dhoop[i]);
            float *st = c.p->c.stats + (c.w * N + i) * 2;
            st[0] = 0.f; st[1] = 0.f;
        }
    }
    F3 ball_at = f3(c.p->start_x, c.p->start_y, 0.f);
    const int32_t off_id = setup_agent_positions(s, c, &ball_at);
    s.set_bpos(ball_at);
    s.fl = 0; s.lta = PH; s.ltt = PH; s.sba = PH; s.sbt = PH; s.spv = 2; s.gin = 0;
    s.bvx = 0.f; s.bvy = 0.f; s.bvz = 0.f;
    if (s.g_1v1 == 1) { s.grab = 1; s.holder = off_id; }
    else { s.grab = 0; s.holder = PH; }
}

// assignInbounder (src/game.cpp:14-53)
template <int N>
BB_HD void assign_inbounder(World<N> &s, F3 ball_pos, int32_t new_team, Q4 orient, bool is_oob)
{
    float assigned = 0.0f;
#pragma unroll
    for (int i = 0; i < N; i++) {
        if (s.team[i] == new_team && assigned == 0.f) {
            assigned = 1.f;
            s.inb[i] = 1;
            s.set_pos(i, ball_pos);
            s.grab = 1; s.holder = AGENT0_ID + i;
            s.has[i] = 1; s.bid[i] = BALL_ID;
            s.set_q(i, orient);
        }
    }
    if (assigned > 0.f) {
        s.g_poss = (float)new_team;
        s.g_inb = 1;
        s.g_inbclk = 5.f;
        if (is_oob) s.g_oob += 1.f;
    }
}

template <int N>
BB_HD int offense_index(const World<N> &s)  // game.cpp:1012-1018, 1072-1078
{
    int off = 0;
#pragma unroll
    for (int i = 1; i < N; i++)
        if ((float)s.team[i] == s.g_poss) off = i;
    return off;
}

// ------------------------------------------------------------------ systems
template <int N>
BB_HD void sys_tick(World<N> &s)  // game.cpp:969-988
{
#pragma unroll
    for (int i = 0; i < N; i++) {
        s.rew[i] = 0.f;
        if (s.rst[i] == 1) { s.done[i] = 1.f; s.step[i] = 0; }
        else { s.done[i] = 0.f; s.step[i] = s.step[i] + 1u; }
        s.cd[i] = maxf(0.f, s.cd[i] - 1.f);
    }
}

template <int N>
BB_HD void sys_action_mask(World<N> &s, uint32_t flags)  // game.cpp:489-533
{
#pragma unroll
    for (int i = 0; i < N; i++) {
        int32_t mv = 1, gr = 1, pa = 0, sh = 0;
        if (s.has[i] == 1) { pa = 1; sh = 1; }
        if (s.g_inb == 1) {
            sh = 0; gr = 0;
            if (s.inb[i] == 1 && s.g_live == 0) mv = 0;
        }
        if (s.cd[i] > 0.f) gr = 0;
        if (!(flags & FLAG_NO_TAG_MASK)) { pa = 0; gr = 0; }
        s.msk[i][0] = mv; s.msk[i][1] = gr; s.msk[i][2] = pa; s.msk[i][3] = sh;
    }
}

// ---- moveAgentSystem (game.cpp:410-486), one agent ---------------------
struct MoveIn {
    int32_t rotate, move, angle, can_move, has;
    Q4 q;
    F3 vel;
    float px, py, max_speed, quickness;
};
struct MoveOut {
    Q4 q;
    F3 vel;
    float px, py;
};

template <int N>
BB_HD MoveIn gather_move(const World<N> &s, int i)
{
    MoveIn m;
    m.rotate = pick_by<N>(i, [&](int j) { return s.act[j][2]; });
    m.move = pick_by<N>(i, [&](int j) { return s.act[j][0]; });
    m.angle = pick_by<N>(i, [&](int j) { return s.act[j][1]; });
    m.can_move = pick_by<N>(i, [&](int j) { return s.msk[j][0]; });
    m.has = pick_by<N>(i, [&](int j) { return s.has[j]; });
    m.q = pick_by<N>(i, [&](int j) { return s.q(j); });
    m.vel = pick_by<N>(i, [&](int j) { return s.vel(j); });
    m.px = pick_by<N>(i, [&](int j) { return s.px[j]; });
    m.py = pick_by<N>(i, [&](int j) { return s.py[j]; });
    m.max_speed = pick_by<N>(i, [&](int j) { return s.attr[j][0]; });
    m.quickness = pick_by<N>(i, [&](int j) { return s.attr[j][1]; });
    return m;
}

BB_HD MoveOut move_one(const MoveIn &in, const Params &p)
{
    MoveOut o;
    // the tables' values first, unconditionally (branch-free selects below)
    const Q4 t0 = sconst(p.turn_q[0]), t1 = sconst(p.turn_q[1]);
    float ts[8], tc[8];
#pragma unroll
    for (int k = 0; k < 8; k++) { ts[k] = sconst(p.mv_sin[k]); tc[k] = sconst(p.mv_cos[k]); }
    o.q = in.q;
    if (in.rotate != 0) o.q = qmul(sel(in.rotate == 1, t0, t1), in.q);
    o.vel = in.vel; o.px = in.px; o.py = in.py;
    if (in.can_move == 0) return o;
    const int32_t m = in.angle;
    float sn = ts[0], cs = tc[0];
#pragma unroll
    for (int k = 1; k < 8; k++) {
        sn = m == k ? ts[k] : sn;
        cs = m == k ? tc[k] : cs;
    }
    if ((uint32_t)m >= 8u) bbm::sincosf_((float)m * ANGLE_STEP, &sn, &cs);
    F3 dv = (f3(sn, -cs, 0.f) * in.quickness) * (float)in.move;
    float maxs = in.max_speed;
    const F3 fw = forward(o.q);
    F3 v = in.vel;
    float d = 0.f;
    if (len2(v) > 1e-6f) d = dot(norm(v), fw);
    if (d < -0.1f) { maxs *= .1f; dv = dv * .1f; }
    else if (d <= 0.8f) { maxs *= .7f; dv = dv * .1f; }
    v = v + dv;
    if (in.has == 1) maxs *= BALL_SLOW;
    if (len(v) > maxs) v = v * (maxs / len(v));
    const float dx = v.x * TS, dy = v.y * TS;
    // the binding's grid is all-empty (src/bindings.cpp:7-11): the wall
    // lookup of game.cpp:472-484 always accepts the move.
    o.px = clampf(in.px + dx, 0.f, p.width);
    o.py = clampf(in.py + dy, 0.f, p.height);
    o.vel = v * .95f;
    return o;
}

template <int N>
BB_HD void apply_move(World<N> &s, int j, const MoveOut &o)
{
    s.set_q(j, o.q); s.set_vel(j, o.vel); s.px[j] = o.px; s.py[j] = o.py;
}

template <int N, class A>
BB_HD void sys_move_agents(World<N> &s, const Ctx &c, const A &ag)
{
    // agent i reads only its own columns
    ag.template each<N>([&](int i) { return move_one(gather_move(s, i), *c.p); },
                        [&](int i, const MoveOut &o) { apply_move(s, i, o); });
}

template <int N>
BB_HD void sys_grab(World<N> &s, const Ctx &c, int i)  // game.cpp:164-239
{
    if (s.msk[i][1] == 0 || s.act[i][3] == 0) return;
    s.cd[i] = 10.f;
    s.act[i][3] = 0;
    if (s.fl == 1) return;
    const int32_t id = AGENT0_ID + i;
    if (s.has[i] == 1 && s.grab == 1 && s.holder == id) {
        s.bid[i] = PH; s.has[i] = 0; s.holder = PH; s.grab = 0;
        return;
    }
    if (len2(s.bpos() - s.pos(i)) <= c.p->grab_le2) {  // len <= 0.3f
        if ((float)s.g_1v1 == 1.f && (float)s.team[i] != s.g_poss) {
            s.reset_now = 1;
            return;
        }
#pragma unroll
        for (int j = 0; j < N; j++)
            if (s.bid[j] == BALL_ID) { s.has[j] = 0; s.bid[j] = PH; s.cd[j] = 62.0f; }
        s.has[i] = 1; s.bid[i] = BALL_ID;
        s.holder = id; s.grab = 1; s.fl = 0;
        s.set_bvel(f3(0.f, 0.f, 0.f));
        s.sba = PH; s.sbt = PH; s.spv = 2;
        s.g_poss = (float)s.team[i];
        s.g_live = 1;
    }
}

template <int N>
BB_HD void sys_pass(World<N> &s, int i)  // game.cpp:243-270
{
    if (s.msk[i][2] == 0 || s.act[i][4] == 0) return;
    if (s.holder == AGENT0_ID + i) {
        s.grab = 0; s.holder = PH;
        s.has[i] = 0; s.bid[i] = PH; s.inb[i] = 0;
        s.set_bvel(rotate(s.q(i), f3(0.f, 0.1f, 0.f)));
        s.g_inb = 0;
    }
}

// ---- shootSystem (game.cpp:273-407), one agent --------------------------
// Agents shoot in creation order and draw 1-3 uniforms each from the world's
// stream; only the ball holder's shot touches the ball, and no agent's shot
// changes what a later agent reads except the stream position.  So agent i
// is computed on its own from the counter after agents 0..i-1's draws.
template <int N>
BB_HD float nearest_opponent(const World<N> &s, int i)  // game.cpp:311-322
{
    const F3 pos = pick_by<N>(i, [&](int j) { return s.pos(j); });
    const int32_t team = pick_by<N>(i, [&](int j) { return s.team[j]; });
    float nd = __builtin_inff();
#pragma unroll
    for (int j = 0; j < N; j++) {
        if (s.team[j] != team) {
            const float dd = len(pos - s.pos(j));
            if (dd < nd) nd = dd;
        }
    }
    return nd;
}

// nearest_opponent(s, i) < 2.0f without a root: some opponent's squared
// distance below Params::near_lt2
template <int N>
BB_HD bool opponent_within_2(const World<N> &s, const Ctx &c, int i)
{
    const F3 pos = pick_by<N>(i, [&](int j) { return s.pos(j); });
    const int32_t team = pick_by<N>(i, [&](int j) { return s.team[j]; });
    bool near = false;
#pragma unroll
    for (int j = 0; j < N; j++)
        if (s.team[j] != team && len2(pos - s.pos(j)) < c.p->near_lt2) near = true;
    return near;
}

template <int N>
BB_HD bool shoots(const World<N> &s, int i)
{
    return s.msk[i][3] != 0 && s.act[i][5] != 0;
}

template <int N>
BB_HD uint32_t shoot_draws(const World<N> &s, const Ctx &c, int i)  // uniforms agent i's shot consumes
{
    if (!shoots(s, i)) return 0u;
    return 1u + (opponent_within_2(s, c, i) ? 1u : 0u) + (s.act[i][0] > 0 ? 1u : 0u);
}

struct ShootOut {
    Q4 q;           // new orientation (shot == 1)
    F3 fs;          // shot direction
    int32_t shot;   // the agent shot this step
    int32_t going;  // the shot goes in
    int32_t value;  // point value of the holder's shot
    int32_t pad;
};

template <int N>
BB_HD ShootOut shoot_one(const World<N> &s, const Ctx &c, int i)
{
    ShootOut o;
    o.q = pick_by<N>(i, [&](int j) { return s.q(j); });
    o.fs = f3(0.f, 0.f, 0.f);
    o.shot = 0; o.going = 0; o.value = 0; o.pad = 0;
    const bool me = pick_by<N>(i, [&](int j) { return shoots(s, j); });
    if (!me) return o;
    uint32_t ctr = s.rng_ctr;
#pragma unroll
    for (int j = 0; j < N - 1; j++)
        if (j < i) ctr += shoot_draws(s, c, j);
    auto draw = [&](float lo, float hi) { return sample_uniform_at(s, c, ctr++, lo, hi); };
    const F3 pos = pick_by<N>(i, [&](int j) { return s.pos(j); });
    const int32_t dhoop = pick_by<N>(i, [&](int j) { return s.dhoop[j]; });
    // attacking hoop: the last hoop (creation order) that is not defended
    F3 target = f3(0.f, 0.f, 0.f);
    float radius = 0.f;
    if (HOOP0_ID != dhoop) { target = hoop_pos<N>(c, 0); radius = HOOP_ZONE; }
    if (HOOP1_ID != dhoop) { target = hoop_pos<N>(c, 1); radius = HOOP_ZONE; }
    const F3 ideal = target - pos;
    const float intended = bbm::atan2f_(ideal.x, ideal.y);
    const float dstd = DIST_DEV * len(ideal);
    const float dev_d = draw(-dstd, dstd);
    float dev_def = 0.0f;
    const float nd = nearest_opponent(s, i);
    if (nd < 2.0f) {
        const float sd = DEF_DEV / (nd + 0.1f);
        dev_def = draw(-sd, sd);
    }
    float dev_v = 0.0f;
    if (pick_by<N>(i, [&](int j) { return s.act[j][0]; }) > 0) {
        const float sv = VEL_DEV * len(pick_by<N>(i, [&](int j) { return s.vel(j); }));
        dev_v = draw(-sv, sv);
    }
    const float dir = intended + ((dev_d + dev_def) + dev_v);
    float sn, cs;
    bbm::sincosf_(dir, &sn, &cs);
    o.fs = f3(sn, cs, 0.f);
    const float along = dot(ideal, o.fs);
    if (!(along < 0.f)) o.going = (len2(ideal) - along * along <= radius * radius) ? 1 : 0;
    o.q = rotation_from_forward(o.fs);
    o.shot = 1;
    if (s.holder == AGENT0_ID + i) o.value = shot_point_value(pos, target, c.p->arc_ge2);
    return o;
}

template <int N>
BB_HD void apply_shoot(World<N> &s, int i, const ShootOut &o)
{
    if (!o.shot) return;
    s.set_q(i, o.q);
    if (s.holder == AGENT0_ID + i) {
        if (o.going == 1) { s.gin = 1; s.g_bask += 1.f; }
        else s.rew[i] -= 1.f;
        s.grab = 0; s.holder = PH;
        s.has[i] = 0; s.bid[i] = PH; s.inb[i] = 0;
        s.set_bvel(o.fs * .1f);
        s.fl = 1;
        s.sba = AGENT0_ID + i; s.sbt = s.team[i]; s.spv = o.value;
        s.lta = AGENT0_ID + i; s.ltt = s.team[i];
    }
}

template <int N, class A>
BB_HD void sys_shoot(World<N> &s, const Ctx &c, const A &ag)
{
    // the stream position after every agent's draws, from the state before
    // the system (apply_shoot changes nothing shoot_draws or shoot_one reads
    // for another agent: only the holder's shot touches ball and possession)
    uint32_t draws = 0;
#pragma unroll
    for (int i = 0; i < N; i++) draws += shoot_draws(s, c, i);
    ag.template each<N>([&](int i) { return shoot_one(s, c, i); },
                        [&](int i, const ShootOut &o) { apply_shoot(s, i, o); });
    s.rng_ctr += draws;
}

template <int N>
BB_HD void sys_move_ball(World<N> &s, const Ctx &c)  // game.cpp:82-125
{
#pragma unroll
    for (int i = 0; i < N; i++)
        if (s.has[i] == 1 && s.grab == 1 && s.holder == AGENT0_ID + i) s.set_bpos(s.pos(i));
    if (len(s.bvel()) == 0.f || s.grab == 1) return;
    const float nx = clampf(s.bx + s.bvx, 0.f, c.p->width);
    const float ny = clampf(s.by + s.bvy, 0.f, c.p->height);
    const float nz = s.bz + s.bvz;
    s.bx = nx; s.by = ny; s.bz = nz;  // empty grid: never a wall (game.cpp:118-124)
}

// ---- updateCurrentShotPercentage (game.cpp:758-809), one agent ---------
template <int N>
BB_HD float shot_pct_one(const World<N> &s, const Ctx &c, int i)
{
    const int32_t has = pick_by<N>(i, [&](int j) { return s.has[j]; });
    if (has == 0) return 0.f;
    const F3 p = pick_by<N>(i, [&](int j) { return s.pos(j); });
    const int32_t team = pick_by<N>(i, [&](int j) { return s.team[j]; });
    const int32_t dhoop = pick_by<N>(i, [&](int j) { return s.dhoop[j]; });
    const F3 hoop = (HOOP0_ID != dhoop) ? hoop_pos<N>(c, 0) : hoop_pos<N>(c, 1);
    const float dh = len(hoop - p);
    float nd = __builtin_inff();
#pragma unroll
    for (int j = 0; j < N; j++) {
        if (s.team[j] != team) {
            const float dd = len(p - s.pos(j));
            if (dd < nd) nd = dd;
        }
    }
    const float ds = DIST_DEV * dh;
    const float fs = DEF_DEV / nd + .0001f;
    const float vs = VEL_DEV * len(pick_by<N>(i, [&](int j) { return s.vel(j); }));
    const float sd = bbm::sqrtf_((ds * ds / 3.f) + (fs * fs / 3.f) + (vs * vs / 3.f));
    const float z = bbm::atanf_(HOOP_ZONE / dh) / sd;
    return (float)bbm::erf_d((double)(z / bbm::sqrtf_(2.f)), c.erf_tab);
}

template <int N, class A>
BB_HD void sys_shot_percentage(World<N> &s, const Ctx &c, const A &ag)
{
    // reads nothing it writes
    ag.template each<N>([&](int i) { return shot_pct_one(s, c, i); }, [&](int i, float v) { s.attr[i][8] = v; });
}

template <int N>
BB_HD void sys_score(World<N> &s, Ctx &c, int h)  // game.cpp:873-953
{
    const F3 hp = hoop_pos<N>(c, h);
    const int32_t hid = h == 0 ? HOOP0_ID : HOOP1_ID;
    const float dx = s.bx - hp.x, dy = s.by - hp.y;
    if (!((dx * dx + dy * dy) <= c.p->hoop_le2 && (float)s.fl == 1.f)) return;  // sqrt(..) <= HOOP_ZONE
    const int32_t pts = s.spv;
    int32_t inb_team = 0;
#pragma unroll
    for (int j = 0; j < N; j++) {
        if (s.dhoop[j] == hid) inb_team = s.team[j];
        if (AGENT0_ID + j == s.sba && c.writer) {
            float *st = c.p->c.stats + (c.w * N + j) * 2;
            st[0] = st[0] + (float)((s.dhoop[j] == hid) ? -s.spv : s.spv);
        }
    }
    F3 spot;
    if (hid == s.g_h0) { s.g_s1 += (float)pts; spot = f3(CMINX, hp.y + INBOUND_DY, 0.f); }
    else { s.g_s0 += (float)pts; spot = f3(CMAXX, hp.y + INBOUND_DY, 0.f); }
    s.g_bask += 1.f;
    s.fl = 0;
    s.set_bvel(f3(0.f, 0.f, 0.f));
    s.sba = PH; s.sbt = PH; s.spv = 2; s.gin = 0;
    if ((float)s.g_1v1 == 0.f) {
        s.set_bpos(spot);
        assign_inbounder(s, spot, inb_team, rotation_from_forward(vec_to_center(c, s.bpos())), false);
    } else {
        s.reset_now = 1;
    }
}

template <int N>
BB_HD void sys_out_of_bounds(World<N> &s, Ctx &c)  // game.cpp:1055-1113
{
    if (!((s.bx < CMINX || s.bx > CMAXX || s.by < CMINY || s.by > CMAXY) && (float)s.g_inb == 0.f)) return;
    if ((float)s.g_1v1 == 1.f) {
        const int off = offense_index(s);
#pragma unroll
        for (int i = 0; i < N; i++)
            if (i == off) s.rew[i] -= 100.f;  // register selects, not a runtime index
        s.reset_now = 1;
        return;
    }
    s.fl = 0;
    s.set_bvel(f3(0.f, 0.f, 0.f));
    s.g_live = 0;
    const int32_t new_team = 1 - s.ltt;
#pragma unroll
    for (int i = 0; i < N; i++) {
        if (s.has[i] == 1 && s.bid[i] == BALL_ID) {
            s.set_pos(i, s.pos(i) + vec_to_center(c, s.pos(i)));
            s.has[i] = 0; s.bid[i] = PH;
        }
    }
    assign_inbounder(s, s.bpos(), new_team, rotation_from_forward(vec_to_center(c, s.bpos())), true);
}

template <int N>
BB_HD void sys_last_touch(World<N> &s, const Ctx &c)  // game.cpp:1034-1051
{
#pragma unroll
    for (int i = 0; i < N; i++)  // len <= AGENT_SIZE
        if (len2(s.bpos() - s.pos(i)) <= c.p->touch_le2) { s.lta = AGENT0_ID + i; s.ltt = s.team[i]; }
}

template <int N>
BB_HD void sys_clock(World<N> &s)  // game.cpp:992-1030
{
    if ((float)s.g_live > 0.5f && s.g_clock > 0.f) { s.g_clock -= TS; s.g_shot -= TS; }
    if ((float)s.g_inb > 0.5f) s.g_inbclk -= TS;
    if (s.g_clock <= 0.f && (float)s.g_live > 0.5f) {
        const int off = offense_index(s);
#pragma unroll
        for (int i = 0; i < N; i++)
            if (i == off) s.rew[i] += 10.f;
        s.reset_now = 1;
    }
    if (s.g_shot < 0.f) s.g_shot = 0.f;
}

template <int N>
BB_HD void sys_inbound_violation(World<N> &s, Ctx &c)  // game.cpp:1116-1157
{
    if (!((float)s.g_inb > 0.5f && s.g_inbclk <= 0.f)) return;
    const int32_t new_team = 1 - (int32_t)s.g_poss;
    int32_t turn_id = PH;
    s.g_live = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        if ((float)s.inb[i] > 0.5f) {
            turn_id = s.bid[i];
            s.inb[i] = 0; s.has[i] = 0; s.bid[i] = PH;
            s.set_pos(i, s.pos(i) + vec_to_center(c, s.pos(i)));
        }
    }
    if (turn_id != PH && turn_id == BALL_ID) {
        s.grab = 0; s.holder = PH;
        assign_inbounder(s, s.bpos(), new_team, rotation_from_forward(vec_to_center(c, s.bpos())), true);
    }
}

// ---- updatePointsWorthSystem (game.cpp:129-161), one agent -------------
template <int N>
BB_HD int32_t points_worth_one(const World<N> &s, const Ctx &c, int i)
{
    // first hoop (creation order) that is not defended; both are never defended at once
    const F3 p = pick_by<N>(i, [&](int j) { return s.pos(j); });
    const int32_t dhoop = pick_by<N>(i, [&](int j) { return s.dhoop[j]; });
    if (HOOP0_ID != dhoop) return shot_point_value(p, hoop_pos<N>(c, 0), c.p->arc_ge2);
    if (HOOP1_ID != dhoop) return shot_point_value(p, hoop_pos<N>(c, 1), c.p->arc_ge2);
    return 2;
}

template <int N, class A>
BB_HD void sys_points_worth(World<N> &s, const Ctx &c, const A &ag)
{
    // reads only pos/dhoop
    ag.template each<N>([&](int i) { return points_worth_one(s, c, i); }, [&](int i, int32_t v) { s.pw[i] = v; });
}

struct Proj { float mn, mx; };
BB_HD Proj project(const F3 (&v)[4], F3 axis)  // helper.cpp:85-100
{
    Proj p; p.mn = dot(v[0], axis); p.mx = p.mn;
#pragma unroll
    for (int k = 1; k < 4; k++) {
        const float d = dot(v[k], axis);
        if (d < p.mn) p.mn = d;
        if (d > p.mx) p.mx = d;
    }
    return p;
}

// Oriented-rectangle SAT contact between agents a < b (game.cpp:537-648).
// Centres farther apart than the two circumscribed circles (+1% + 1 cm):
// the rectangles are disjoint with a margin far above float rounding, so the
// SAT test below finds a separating axis and changes nothing -- skip it.
constexpr float COLLIDE_CULL = (float)((2.0 * 1.01) * 0.2202504256522561 + 0.01);  // circumradius of 0.429 x 0.1
static_assert(HALF_SHOULDER > 0.2144f && HALF_SHOULDER < 0.2146f && HALF_DEPTH > 0.0499f && HALF_DEPTH < 0.0501f,
              "COLLIDE_CULL assumes the 0.429 x 0.1 agent rectangle");

template <int N>
BB_HD bool collide_near(const World<N> &s, int a, int b)
{
    const float dx = s.px[b] - s.px[a], dy = s.py[b] - s.py[a];
    return !(dx * dx + dy * dy > COLLIDE_CULL * COLLIDE_CULL);
}

// Returns whether the pair collided (positions changed).
template <int N>
BB_HD bool collide_pair(World<N> &s, int a, int b)
{
    if (!collide_near(s, a, b)) return false;
    const F3 ca = s.pos(a), fa = forward(s.q(a));
    const F3 ra = f3(fa.y, -fa.x, 0.f);
    const F3 hwa = ra * HALF_SHOULDER, hda = fa * HALF_DEPTH;
    const F3 va[4] = {(ca - hda) + hwa, (ca - hda) - hwa, (ca + hda) - hwa, (ca + hda) + hwa};
    const F3 cb = s.pos(b), fb = forward(s.q(b));
    const F3 rb = f3(fb.y, -fb.x, 0.f);
    const F3 hwb = rb * HALF_SHOULDER, hdb = fb * HALF_DEPTH;
    const F3 vb[4] = {(cb - hdb) + hwb, (cb - hdb) - hwb, (cb + hdb) - hwb, (cb + hdb) + hwb};
    const F3 axes[4] = {norm(ra), norm(fa), norm(rb), norm(fb)};
    float min_ov = 3.40282347e+38f;
    F3 mtv = f3(0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const Proj pa = project(va, axes[k]), pb = project(vb, axes[k]);
        if (!(pa.mx > pb.mn && pb.mx > pa.mn)) return false;  // separating axis
        const float ov = minf(pa.mx, pb.mx) - maxf(pa.mn, pb.mn);
        if (ov < min_ov) { min_ov = ov; mtv = axes[k]; }
    }
    if (s.g_poss == (float)s.team[a]) {
        s.rew[a] -= 10.f;
        s.rew[b] += 10.f;
        s.reset_now = 1;
    }
    F3 corr = mtv;
    if (dot(cb - ca, corr) < 0.f) corr = -corr;
    s.set_pos(a, s.pos(a) - (corr * min_ov) * 0.5f);
    s.set_pos(b, s.pos(b) + (corr * min_ov) * 0.5f);
    return true;
}

// agentCollisionSystem over the pairs a < b in order.  With the world in
// indexable memory (N >= LDS_WORLD_MIN_N) the cull tests of all pairs run
// first, agent a's lane testing pairs (a, b > a) on the positions as they
// are before any pair resolves; pairs are then visited in order through the
// close ones only, until a pair collides: its agents moved, so from the next
// pair on every pair is tested again on the current positions (the plain
// serial loop).  Before the first collision no position has changed, so a
// pair that was far then is far when its turn comes: the same pairs collide,
// in the same order, as in the serial loop.
template <int N, class A = EachAgent>
BB_HD void sys_collisions(World<N> &s, const A &ag = A())
{
    if constexpr (N < LDS_WORLD_MIN_N) {
#pragma unroll
        for (int a = 0; a < N; a++)
#pragma unroll
            for (int b = a + 1; b < N; b++) collide_pair(s, a, b);
    } else {
        uint32_t near[N];  // bit b of near[a]: pair (a, b), b > a, within the cull distance
        ag.all([&](int a) {
            uint32_t m = 0;
            for (int b = a + 1; b < N; b++)
                if (collide_near(s, a, b)) m |= 1u << b;
            return m;
        }, near);
        for (int a = 0; a < N; a++) {
            uint32_t m = near[a];
            while (m) {
                const int b = __builtin_ctz(m);
                m &= m - 1;
                if (collide_pair(s, a, b)) {  // positions changed: the rest as the serial loop
                    for (int b2 = b + 1; b2 < N; b2++) collide_pair(s, a, b2);
                    for (int a2 = a + 1; a2 < N; a2++)
                        for (int b2 = a2 + 1; b2 < N; b2++) collide_pair(s, a2, b2);
                    return;
                }
            }
        }
    }
}

// ---- hardCodeDefenseSystem (game.cpp:651-755), one agent --------------
struct DefOut {
    int32_t act[4];  // move, moveAngle, rotate, grab
    F3 target;       // Attributes.currentTargetPosition
};

template <int N>
BB_HD DefOut defense_one(const World<N> &s, const Ctx &c, int i)
{
    DefOut o;
#pragma unroll
    for (int q = 0; q < 4; q++) o.act[q] = pick_by<N>(i, [&](int j) { return s.act[j][q]; });
    o.target = pick_by<N>(i, [&](int j) { return s.target(j); });
    const int32_t team = pick_by<N>(i, [&](int j) { return s.team[j]; });
    if (s.g_poss == (float)team) { o.act[0] = 0; return o; }
    o.act[3] = 1;
    const int32_t dhoop = pick_by<N>(i, [&](int j) { return s.dhoop[j]; });
    F3 guard = f3(0.f, 0.f, 0.f);
    bool found = false;
#pragma unroll
    for (int j = 0; j < N; j++) {
        if (s.has[j] == 1 && !found) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                if (dhoop == (h == 0 ? HOOP0_ID : HOOP1_ID)) {
                    const F3 hd = hoop_pos<N>(c, h) - s.pos(j);
                    guard = (len2(hd) > 1e-6f) ? s.pos(j) + norm(hd) * GUARD : s.pos(j);
                    found = true;
                }
            }
        }
    }
    if (!found) { o.act[0] = 0; return o; }
    const F3 cur = o.target;
    const float react = pick_by<N>(i, [&](int j) { return s.attr[j][4]; });
    o.target = cur + (guard - cur) * (react * TS);
    const F3 mv = o.target - pick_by<N>(i, [&](int j) { return s.pos(j); });
    if (len2(mv) < 0.01f) { o.act[0] = 0; return o; }
    // argmax over the 8 move directions of game.cpp:713-722 (first max wins)
    const F3 desired = norm(mv);
    const float diag = 1.0f / bbm::sqrtf_(2.f);
    const float dots[8] = {
        dot(desired, f3(0.f * 1.f, -1.f * 1.f, 0.f)), dot(desired, f3(1.f * diag, -1.f * diag, 0.f * diag)),
        dot(desired, f3(1.f * 1.f, 0.f * 1.f, 0.f)), dot(desired, f3(1.f * diag, 1.f * diag, 0.f * diag)),
        dot(desired, f3(0.f * 1.f, 1.f * 1.f, 0.f)), dot(desired, f3(-1.f * diag, 1.f * diag, 0.f * diag)),
        dot(desired, f3(-1.f * 1.f, 0.f * 1.f, 0.f)), dot(desired, f3(-1.f * diag, -1.f * diag, 0.f * diag))};
    float maxd = -2.f;
    int32_t best = 0;
#pragma unroll
    for (int k = 0; k < 8; k++)
        if (dots[k] > maxd) { maxd = dots[k]; best = k; }
    o.act[0] = 1;
    o.act[1] = best;
    const F3 fw = forward(pick_by<N>(i, [&](int j) { return s.q(j); }));
    const float cosang = clampf(dot(fw, norm(mv)), -1.f, 1.f);
    const bool turn = c.p->rot_exact ? ((float)bbm::acos_d((double)cosang) > PI_OVER_8)
                                     : (cosang < c.p->rot_thresh);
    if (turn) {
        const float cr = fw.x * mv.y - fw.y * mv.x;
        o.act[2] = cr < 0.f ? -1 : (cr > 0.f ? 1 : 0);
    } else {
        o.act[2] = 0;
    }
    return o;
}

template <int N>
BB_HD void apply_defense(World<N> &s, int j, const DefOut &o)
{
#pragma unroll
    for (int q = 0; q < 4; q++) s.act[j][q] = o.act[q];
    s.set_target(j, o.target);
}

template <int N, class A>
BB_HD void sys_defense(World<N> &s, const Ctx &c, const A &ag)
{
    // agent i reads only fields no other agent's defence writes
    ag.template each<N>([&](int i) { return defense_one(s, c, i); },
                        [&](int i, const DefOut &o) { apply_defense(s, i, o); });
}

// ---- rewardSystem (game.cpp:811-870), one agent ------------------------
template <int N>
BB_HD float reward_one(const World<N> &s, int i, int32_t id)
{
    // `other` = the last agent (creation order) that is not self
    const F3 p = pick_by<N>(i, [&](int j) { return s.pos(j); });
    const F3 po = pick_by<N>(i, [&](int j) { return s.pos(j == N - 1 ? N - 2 : N - 1); });
    const float dist = len(po - p);
    float r = pick_by<N>(i, [&](int j) { return s.rew[j]; });
    const int32_t team = pick_by<N>(i, [&](int j) { return s.team[j]; });
    if ((float)team == s.g_poss) {
        if (s.g_clock > 5.f) {
            if (s.sba == id && s.gin == 1) r += (float)s.spv;
            else if (s.sba == id && s.gin == 0 && s.fl == 1) r -= 1.f;
            r += pick_by<N>(i, [&](int j) { return s.attr[j][8]; });
        }
    } else {
        r -= 1.f;
        r = (float)((double)r + bbm::exp_d((double)(-0.4f * dist)));
    }
    return r;
}

template <int N>
BB_HD void sys_reward_agent(World<N> &s, int i, int32_t id)
{
    s.rew[i] = reward_one(s, i, id);
}

template <int N>
BB_HD void sys_reward(World<N> &s)
{
#pragma unroll
    for (int i = 0; i < N; i++) sys_reward_agent(s, i, AGENT0_ID + i);
}

// ------------------------------------------------------------------ observations
// fillObservationsSystem (game.cpp:1175-1461).  Values are produced in row
// order through a sink; with N a compile-time constant every index below
// folds to a constant and the sink becomes straight-line float4 stores.
struct RowSink {
    float *row;
    float b0, b1, b2, b3;
    int idx;
    BB_HD void put(float v)
    {
        switch (idx & 3) {
        case 0: b0 = v; break;
        case 1: b1 = v; break;
        case 2: b2 = v; break;
        default: b3 = v; store_f4(row + (idx & ~3), b0, b1, b2, b3); break;
        }
        idx++;
    }
    BB_HD void put3(F3 v) { put(v.x); put(v.y); put(v.z); }
    BB_HD void put4(Q4 q) { put(q.w); put(q.x); put(q.y); put(q.z); }
    // zero-fill up to the next 4-float boundary (the row tail beyond is
    // zero from construction and never written non-zero)
    BB_HD void finish() { while (idx & 3) put(0.f); }
};

// Runtime-indexed sink for the non-canonical team layouts (any Team edits
// that leave a slot empty or overfull): scalar stores over the whole row.
struct SlowRowSink {
    float *row;
    int idx;
    BB_HD void put(float v) { row[idx++] = v; }
    BB_HD void put3(F3 v) { put(v.x); put(v.y); put(v.z); }
    BB_HD void put4(Q4 q) { put(q.w); put(q.x); put(q.y); put(q.z); }
};

// The 31 values of an agent block that depend only on agent j and the hoop it
// is measured against (game.cpp:1293-1322 for self, :1343-1372 / :1384-1421
// for teammates / opponents): orientation, forward, velocity direction,
// speed, facing dot, acceleration factor, hoop direction + distance, ball
// direction + distance, inbounding, cooldown, 6 attributes, pointsWorth,
// hasBall.
template <int N, class Sink>
BB_HD void emit_intrinsic(const World<N> &s, Sink &o, int j, F3 hoop)
{
    const F3 pj = s.pos(j);
    const Q4 qj = s.q(j);
    o.put4(qj);
    const F3 fw = forward(qj);
    o.put3(fw);
    const F3 v = s.vel(j);
    const bool moving = len2(v) > 1e-6f;
    o.put3(moving ? norm(v) : f3(0.f, 0.f, 0.f));
    o.put(len(v));
    const float d = moving ? dot(norm(v), fw) : 0.f;
    o.put(d);
    o.put(d <= 0.8f ? 0.1f : 1.f);
    const F3 th = hoop - pj;
    const float dh = len(th);
    o.put3(dh > 1e-6f ? norm(th) : f3(0.f, 0.f, 0.f));
    o.put(dh);
    const F3 tb = s.bpos() - pj;
    const float db = len(tb);
    o.put3(db > 1e-6f ? norm(tb) : f3(0.f, 0.f, 0.f));
    o.put(db);
    o.put((float)s.inb[j]);
    o.put(s.cd[j]);
    o.put(s.attr[j][0]); o.put(s.attr[j][1]); o.put(s.attr[j][2]);
    o.put(s.attr[j][3]); o.put(s.attr[j][4]); o.put(s.attr[j][8]);
    o.put((float)s.pw[j]);
    o.put((float)s.has[j]);
}
constexpr int INTRINSIC = 31;

// A fixed-size buffer sink (compile-time indices fold it into registers).
template <int LEN>
struct ArraySink {
    float v[LEN];
    int idx;
    BB_HD void put(float x) { v[idx++] = x; }
    BB_HD void put3(F3 a) { put(a.x); put(a.y); put(a.z); }
    BB_HD void put4(Q4 q) { put(q.w); put(q.x); put(q.y); put(q.z); }
};

template <int N, class Sink>
BB_HD void obs_agent_block(const World<N> &s, Sink &o, int j, F3 self_pos, F3 hoop)
{
    const F3 pj = s.pos(j), to = pj - self_pos;
    o.put3(pj);
    o.put3(len2(to) > 1e-6f ? norm(to) : f3(0.f, 0.f, 0.f));
    o.put(len(to));
    emit_intrinsic(s, o, j, hoop);
}

template <int N>
BB_HD F3 attacking_hoop(const World<N> &s, const Ctx &c, int a)  // game.cpp:1284
{
    return (HOOP0_ID != s.dhoop[a]) ? hoop_pos<N>(c, 0) : hoop_pos<N>(c, 1);
}

// Game context + egocentric score + ball + hoops (obs 0-22, game.cpp:1256-1287)
template <int N, class Sink>
BB_HD void obs_context(const World<N> &s, const Ctx &c, Sink &o, int a, F3 *att, F3 *dfn)
{
    o.put(s.g_clock); o.put(s.g_shot); o.put(s.g_period);
    o.put((float)s.g_inb); o.put(s.g_inbclk);
    o.put(s.team[a] == 0 ? s.g_s0 : s.g_s1);
    o.put(s.team[a] == 0 ? s.g_s1 : s.g_s0);
    o.put3(s.bpos()); o.put3(s.bvel());
    o.put((float)s.grab); o.put((float)s.fl); o.put((float)s.spv); o.put((float)s.ltt);
    *att = attacking_hoop(s, c, a);
    *dfn = (HOOP0_ID == s.dhoop[a]) ? hoop_pos<N>(c, 0) : hoop_pos<N>(c, 1);
    o.put3(*att); o.put3(*dfn);
}

template <int N, class Sink>
BB_HD void obs_header(const World<N> &s, const Ctx &c, Sink &o, int a, F3 *att, F3 *dfn)
{
    obs_context(s, c, o, a, att, dfn);
    // self block (23..60): position, 4 zeros, then the intrinsic values
    o.put3(s.pos(a));
    o.put3(f3(0.f, 0.f, 0.f));
    o.put(0.f);
    emit_intrinsic(s, o, a, *att);
}

template <int N>
BB_HD int32_t inbounder_id(const World<N> &s)
{
    int32_t id = -1;
#pragma unroll
    for (int i = 0; i < N; i++) if ((float)s.inb[i] > 0.5f) id = AGENT0_ID + i;
    return id;
}

// true when every other agent fills a slot: exactly N/2-1 teammates and N/2
// opponents (always the case for the generated i % 2 teams)
template <int N>
BB_HD bool canonical_slots(const World<N> &s, int a)
{
    int mates = 0, opps = 0;
#pragma unroll
    for (int j = 0; j < N; j++) {
        if (j == a) continue;
        if (s.team[j] == s.team[a]) mates++; else opps++;
    }
    return mates == N / 2 - 1 && opps == N / 2;
}

template <int N, class Sink>
BB_HD void emit_row_fast(const World<N> &s, const Ctx &c, int a, Sink &o, int32_t ib)
{
    F3 att, dfn;
    obs_header(s, c, o, a, &att, &dfn);
    const F3 p = s.pos(a);
#pragma unroll
    for (int j = 0; j < N; j++) {
        if (j == a) continue;
        obs_agent_block(s, o, j, p, s.team[j] == s.team[a] ? att : dfn);
    }
    // one-hot vectors over agents in creation order (absolute ids)
#pragma unroll
    for (int j = 0; j < N; j++) o.put(AGENT0_ID + j == s.holder ? 1.f : 0.f);
#pragma unroll
    for (int j = 0; j < N; j++) o.put(AGENT0_ID + j == ib ? 1.f : 0.f);
    o.finish();
}

template <int N>
BB_HD void fill_obs_fast(const World<N> &s, const Ctx &c, int a, float *row, int32_t ib)
{
    RowSink o;
    o.row = row; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
    emit_row_fast(s, c, a, o, ib);
}

// Observation rows of every agent of a world with each agent's intrinsic
// block computed once (canonical layouts in which the hoop an observer
// measures agent j against is j's own attacking hoop -- always the case for
// the generated teams): bit-identical to fill_obs_fast per agent.
template <int N>
BB_HD bool obs_sharable(const World<N> &s)
{
#pragma unroll
    for (int a = 0; a < N; a++) {
        if (!canonical_slots(s, a)) return false;
        const bool att0_a = HOOP0_ID != s.dhoop[a];
#pragma unroll
        for (int j = 0; j < N; j++) {
            if (j == a) continue;
            // observer a measures j against a's attacking hoop if j is a
            // teammate, else a's defending hoop; j's own attacking hoop:
            const bool chosen0 = (s.team[j] == s.team[a]) ? att0_a : (HOOP0_ID == s.dhoop[a]);
            if (chosen0 != (HOOP0_ID != s.dhoop[j])) return false;
        }
    }
    return true;
}

template <int N>
struct SharedObs {
    ArraySink<INTRINSIC> intr[N];
    F3 rdir[N][N];   // direction from a to j (0 vector below the 1e-6 threshold)
    float rlen[N][N];
};

template <int N>
BB_HD void shared_obs_prepare(const World<N> &s, const Ctx &c, SharedObs<N> &sh)
{
#pragma unroll
    for (int j = 0; j < N; j++) {
        sh.intr[j].idx = 0;
        emit_intrinsic(s, sh.intr[j], j, attacking_hoop(s, c, j));
    }
#pragma unroll
    for (int a = 0; a < N; a++)
#pragma unroll
        for (int j = a + 1; j < N; j++) {
            const F3 to = s.pos(j) - s.pos(a), back = s.pos(a) - s.pos(j);
            const float l2 = len2(to);                        // == len2(back) exactly
            const bool nz = l2 > 1e-6f;
            const float r = 1.0f / bbm::sqrtf_(l2);        // the factor norm() applies
            sh.rdir[a][j] = nz ? to * r : f3(0.f, 0.f, 0.f);
            sh.rdir[j][a] = nz ? back * r : f3(0.f, 0.f, 0.f);  // not -(to * r): +0 stays +0
            sh.rlen[a][j] = sh.rlen[j][a] = bbm::sqrtf_(l2);
        }
}

template <int N, class Sink>
BB_HD void emit_row_shared(const World<N> &s, const Ctx &c, const SharedObs<N> &sh, int a, Sink &o, int32_t ib)
{
    F3 att, dfn;
    obs_context(s, c, o, a, &att, &dfn);
    o.put3(s.pos(a));
    o.put3(f3(0.f, 0.f, 0.f));
    o.put(0.f);
#pragma unroll
    for (int q = 0; q < INTRINSIC; q++) o.put(sh.intr[a].v[q]);
#pragma unroll
    for (int j = 0; j < N; j++) {
        if (j == a) continue;
        o.put3(s.pos(j));
        o.put3(sh.rdir[a][j]);
        o.put(sh.rlen[a][j]);
#pragma unroll
        for (int q = 0; q < INTRINSIC; q++) o.put(sh.intr[j].v[q]);
    }
#pragma unroll
    for (int j = 0; j < N; j++) o.put(AGENT0_ID + j == s.holder ? 1.f : 0.f);
#pragma unroll
    for (int j = 0; j < N; j++) o.put(AGENT0_ID + j == ib ? 1.f : 0.f);
    o.finish();
}

// Row of observer `a` (a runtime index: the world lives in memory that takes
// indexed access, e.g. LDS) with every put at a compile-time position: the
// other agents in creation order are view slots 1..N-1.  intr(j, q) is value
// q of agent j's intrinsic block measured against j's own attacking hoop;
// with share (obs_sharable) those are used for every agent, otherwise the
// other agents' blocks are recomputed against the observer's hoops
// (bit-identical to emit_row_fast for canonical slot layouts).
template <int N, class Sink, class IntrOf>
BB_HD void emit_row_view(const World<N> &s, const Ctx &c, int a, IntrOf intr, bool share, Sink &o, int32_t ib)
{
    F3 att, dfn;
    obs_context(s, c, o, a, &att, &dfn);
    const F3 p = s.pos(a);
    o.put3(p);
    o.put3(f3(0.f, 0.f, 0.f));
    o.put(0.f);
#pragma unroll
    for (int q = 0; q < INTRINSIC; q++) o.put(intr(a, q));
#pragma unroll
    for (int t = 1; t < N; t++) {
        const int j = view_source<N>(t, a);
        const F3 pj = s.pos(j), to = pj - p;
        const float l2 = len2(to);
        const float r = 1.0f / bbm::sqrtf_(l2);  // the factor norm() applies
        o.put3(pj);
        o.put3(l2 > 1e-6f ? to * r : f3(0.f, 0.f, 0.f));
        o.put(bbm::sqrtf_(l2));
        if (share) {
#pragma unroll
            for (int q = 0; q < INTRINSIC; q++) o.put(intr(j, q));
        } else {
            emit_intrinsic(s, o, j, s.team[j] == s.team[a] ? att : dfn);
        }
    }
#pragma unroll
    for (int j = 0; j < N; j++) o.put(AGENT0_ID + j == s.holder ? 1.f : 0.f);
#pragma unroll
    for (int j = 0; j < N; j++) o.put(AGENT0_ID + j == ib ? 1.f : 0.f);
    o.finish();
}

template <int N, class Sink>
BB_HD void emit_row_slow(const World<N> &s, const Ctx &c, int a, Sink &o, int32_t ib)
{
    F3 att, dfn;
    obs_header(s, c, o, a, &att, &dfn);
    const F3 p = s.pos(a);
    int mates = 0, opps = 0;
    const int max_mates = N / 2 - 1, max_opps = N / 2;
    for (int j = 0; j < N; j++) {
        if (j == a) continue;
        if (s.team[j] == s.team[a]) {
            if (mates < max_mates) { obs_agent_block(s, o, j, p, att); mates++; }
        } else {
            if (opps < max_opps) { obs_agent_block(s, o, j, p, dfn); opps++; }
        }
    }
    for (int k = mates; k < max_mates; k++) for (int z = 0; z < 37; z++) o.put(0.f);
    for (int k = opps; k < max_opps; k++) for (int z = 0; z < 37; z++) o.put(0.f);
    for (int j = 0; j < N; j++) o.put(AGENT0_ID + j == s.holder ? 1.f : 0.f);
    for (int j = 0; j < N; j++) o.put(AGENT0_ID + j == ib ? 1.f : 0.f);
    for (; o.idx < obs_width(N); ) o.put(0.f);
}

template <int N>
BB_HD void fill_obs_slow(const World<N> &s, const Ctx &c, int a, float *row, int32_t ib)
{
    SlowRowSink o;
    o.row = row; o.idx = 0;
    emit_row_slow(s, c, a, o, ib);
}

template <int N>
BB_HD void sys_fill_obs(const World<N> &s, const Ctx &c)
{
    const int32_t ib = inbounder_id(s);
    if (obs_sharable(s)) {
        SharedObs<N> sh;
        shared_obs_prepare(s, c, sh);
#pragma unroll
        for (int a = 0; a < N; a++) {
            RowSink o;
            o.row = c.p->c.obs + (c.w * N + a) * (int64_t)obs_width(N);
            o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
            emit_row_shared(s, c, sh, a, o, ib);
        }
        return;
    }
#pragma unroll
    for (int a = 0; a < N; a++) {
        float *row = c.p->c.obs + (c.w * N + a) * (int64_t)obs_width(N);
        if (canonical_slots(s, a)) fill_obs_fast(s, c, a, row, ib);
        else fill_obs_slow(s, c, a, row, ib);
    }
}

// ------------------------------------------------------------------ one step
// Systems 1-17 (everything before fillObservations).  Timing attribution
// only (bb_diag_time): `skip` leaves out the systems whose bit (1 << system
// number) is set; `dup` runs them a second time on a copy of the world whose
// result is dropped (c.p->diag_keep is 0 at run time), so the added time is
// the system's own cost on the unchanged trajectory.  The game passes 0 for
// both and the tests fold away.
template <int N, class A = EachAgent>
BB_HD void step_world_pre_obs(World<N> &s, Ctx &c, const A &ag = A(), uint32_t skip = 0, uint32_t dup = 0)
{
    const uint32_t flags = c.p->flags;
#define BB_RUN(bit, stmt)                                                   \
    if (!(skip & (1u << (bit)))) { stmt; }                                  \
    if (dup & (1u << (bit))) {                                              \
        World<N> s_dup = s;                                                 \
        {                                                                   \
            World<N> &s = s_dup;                                            \
            stmt;                                                           \
        }                                                                   \
        if (c.p->diag_keep) s = s_dup;                                      \
    }
    ag.mark(1);
    BB_RUN(1, sys_tick(s))
    BB_RUN(2, sys_action_mask(s, flags))
    BB_RUN(3, sys_move_agents(s, c, ag))
    ag.mark(2);
    BB_RUN(4, for (int i = 0; i < N; i++) sys_grab(s, c, i))
    BB_RUN(5, for (int i = 0; i < N; i++) sys_pass(s, i))
    BB_RUN(6, sys_shoot(s, c, ag))
    ag.mark(3);
    BB_RUN(7, sys_move_ball(s, c))
    BB_RUN(8, sys_shot_percentage(s, c, ag))
    BB_RUN(9, sys_score(s, c, 0); sys_score(s, c, 1))   // hoop 0, then hoop 1
    ag.mark(4);
    BB_RUN(10, sys_out_of_bounds(s, c))
    BB_RUN(11, sys_last_touch(s, c))
    BB_RUN(12, sys_clock(s))
    BB_RUN(13, sys_inbound_violation(s, c))
    ag.mark(5);
    BB_RUN(14, if (s.reset_now != 0) { reset_world(s, c); s.reset_now = 0; })  // resetSystem
    ag.mark(6);
    BB_RUN(15, sys_points_worth(s, c, ag))
    BB_RUN(16, sys_collisions(s, ag))
    BB_RUN(17, sys_defense(s, c, ag))
#undef BB_RUN
}

template <int N>
BB_HD void step_world(World<N> &s, Ctx &c)
{
    step_world_pre_obs(s, c);                      // 1-17
    sys_reward(s);                                 // 19 (reads nothing fillObservations writes)
    sys_fill_obs(s, c);                            // 18
}

// ------------------------------------------------------------------ agent views
// Copy of `s` with agent k in slot 0 and the other agents after it in
// creation order (k runtime, every array index compile-time: register
// selects, no scratch).  Systems that read "self" and "the others in
// creation order" give identical results on the view's slot 0.
template <class T, int N>
BB_HD T pick(const T (&a)[N], int idx)
{
    T r = a[0];
#pragma unroll
    for (int i = 1; i < N; i++) r = sel(idx == i, a[i], r);
    return r;
}


// INV: the inverse map -- v from agent k's view back to creation order.
template <int N, bool INV = false>
BB_HD void agent_view(const World<N> &s, World<N> &v, int k)
{
    v = s;
#pragma unroll
    for (int j = 0; j < N; j++) {
        const int src = INV ? view_slot<N>(j, k) : view_source<N>(j, k);
#define BB_V(f) v.f[j] = pick(s.f, src);
        BB_V(rst) BB_V(cd) BB_V(px) BB_V(py) BB_V(pz) BB_V(rew) BB_V(done) BB_V(step)
        BB_V(has) BB_V(bid) BB_V(pw) BB_V(qw) BB_V(qx) BB_V(qy) BB_V(qz) BB_V(inb) BB_V(allow)
        BB_V(team) BB_V(dhoop) BB_V(vx) BB_V(vy) BB_V(vz)
#undef BB_V
#pragma unroll
        for (int q = 0; q < 6; q++) {
            int32_t col[N];
#pragma unroll
            for (int i = 0; i < N; i++) col[i] = s.act[i][q];
            v.act[j][q] = pick(col, src);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int32_t col[N];
#pragma unroll
            for (int i = 0; i < N; i++) col[i] = s.msk[i][q];
            v.msk[j][q] = pick(col, src);
        }
#pragma unroll
        for (int q = 0; q < 10; q++) {
            float col[N];
#pragma unroll
            for (int i = 0; i < N; i++) col[i] = s.attr[i][q];
            v.attr[j][q] = pick(col, src);
        }
    }
}

// ------------------------------------------------------------------ load/store
template <int N>
BB_HD void load_world(World<N> &s, const Params &p, int64_t w)
{
    const Columns &c = p.c;
    {
        uint32_t g[14];
        load_words<14>(c.game_state, w, g);
        s.g_inb = (int32_t)g[0]; s.g_live = (int32_t)g[1]; s.g_period = bitsf(g[2]); s.g_poss = bitsf(g[3]);
        s.g_h0 = (int32_t)g[4]; s.g_s0 = bitsf(g[5]); s.g_h1 = (int32_t)g[6]; s.g_s1 = bitsf(g[7]);
        s.g_clock = bitsf(g[8]); s.g_shot = bitsf(g[9]); s.g_bask = bitsf(g[10]); s.g_oob = bitsf(g[11]);
        s.g_inbclk = bitsf(g[12]); s.g_1v1 = (int32_t)g[13];
    }
    s.reset_now = c.world_clock[w];
    s.rng_ctr = c.rng_counter[w];
    {
        uint32_t r[N], a[6 * N], pos[3 * N], ps[3 * N], q[4 * N], v[3 * N], cd[N], st[N], ib[2 * N];
        uint32_t at[10 * N];
        load_words<N>(c.reset, w, r);
        load_words<6 * N>(c.action, w, a);
        load_words<3 * N>(c.agent_pos, w, pos);
        load_words<3 * N>(c.possession, w, ps);
        load_words<4 * N>(c.orientation, w, q);
        load_words<3 * N>(c.agent_vel, w, v);
        load_words<N>(c.cooldown, w, cd);
        load_words<N>(c.cur_step, w, st);
        load_words<2 * N>(c.inbounding, w, ib);
        load_words<10 * N>(c.attributes, w, at);
#pragma unroll
        for (int i = 0; i < N; i++) {
            s.rst[i] = (int32_t)r[i];
#pragma unroll
            for (int k = 0; k < 6; k++) s.act[i][k] = (int32_t)a[6 * i + k];
            s.px[i] = bitsf(pos[3 * i]); s.py[i] = bitsf(pos[3 * i + 1]); s.pz[i] = bitsf(pos[3 * i + 2]);
            s.has[i] = (int32_t)ps[3 * i]; s.bid[i] = (int32_t)ps[3 * i + 1]; s.pw[i] = (int32_t)ps[3 * i + 2];
            s.qw[i] = bitsf(q[4 * i]); s.qx[i] = bitsf(q[4 * i + 1]); s.qy[i] = bitsf(q[4 * i + 2]); s.qz[i] = bitsf(q[4 * i + 3]);
            s.vx[i] = bitsf(v[3 * i]); s.vy[i] = bitsf(v[3 * i + 1]); s.vz[i] = bitsf(v[3 * i + 2]);
            s.cd[i] = bitsf(cd[i]);
            s.step[i] = st[i];
            s.inb[i] = (int32_t)ib[2 * i]; s.allow[i] = (int32_t)ib[2 * i + 1];
#pragma unroll
            for (int k = 0; k < 10; k++) s.attr[i][k] = bitsf(at[10 * i + k]);
            const uint32_t *t = c.team + (w * N + i) * 5;
            s.team[i] = (int32_t)t[0];
            s.dhoop[i] = (int32_t)t[4];
            // Reward and Done are rewritten by tick before any read; ActionMask
            // by actionMaskSystem: none of the three is loaded.
            s.rew[i] = 0.f; s.done[i] = 0.f;
#pragma unroll
            for (int k = 0; k < 4; k++) s.msk[i][k] = 0;
        }
    }
    {
        const float *bp = c.ball_pos + w * 3, *bv = c.ball_vel + w * 3;
        s.bx = bp[0]; s.by = bp[1]; s.bz = bp[2];
        s.bvx = bv[0]; s.bvy = bv[1]; s.bvz = bv[2];
        const int32_t *ph = c.ball_physics + w * 7;
        s.fl = ph[0]; s.lta = ph[1]; s.ltt = ph[2]; s.sba = ph[3]; s.sbt = ph[4]; s.spv = ph[5]; s.gin = ph[6];
        uint32_t gb[2];
        load_words<2>(c.ball_grabbed, w, gb);
        s.grab = (int32_t)gb[0]; s.holder = (int32_t)gb[1];
    }
}

// Event-only words (SURVEY.md 8(d) leaves them out of the per-step traffic):
// GameState except the two clocks, BallPhysics, Grabbed, WorldClock, the RNG
// counter; per agent Reset, Inbounding and the constant attributes (0-4, 9).
// Snapshotted right after the load, they let the store phase rewrite such a
// column only when the step changed it -- memory still holds the loaded
// words, so skipping the store is exact.
struct OrigAgent {
    int32_t rst, inb, allow;
    uint32_t attr[6];  // attributes 0-4, 9
};
struct WorldOrig {
    uint32_t game[14];
    uint32_t phys[7], grab[2], clock, rng;
};
template <int N>
struct Orig : WorldOrig {
    OrigAgent ag[N];
};
template <int N>
BB_HD WorldOrig world_orig(const Orig<N> &o) { return o; }
template <int N>
BB_HD void set_world_orig(Orig<N> &o, const WorldOrig &w) { (WorldOrig &)o = w; }

template <int N>
BB_HD void game_words(const World<N> &s, uint32_t (&g)[14])
{
    g[0] = (uint32_t)s.g_inb; g[1] = (uint32_t)s.g_live; g[2] = fbits(s.g_period); g[3] = fbits(s.g_poss);
    g[4] = (uint32_t)s.g_h0; g[5] = fbits(s.g_s0); g[6] = (uint32_t)s.g_h1; g[7] = fbits(s.g_s1);
    g[8] = fbits(s.g_clock); g[9] = fbits(s.g_shot); g[10] = fbits(s.g_bask); g[11] = fbits(s.g_oob);
    g[12] = fbits(s.g_inbclk); g[13] = (uint32_t)s.g_1v1;
}
template <int N>
BB_HD void phys_words(const World<N> &s, uint32_t (&ph)[7])
{
    ph[0] = (uint32_t)s.fl; ph[1] = (uint32_t)s.lta; ph[2] = (uint32_t)s.ltt; ph[3] = (uint32_t)s.sba;
    ph[4] = (uint32_t)s.sbt; ph[5] = (uint32_t)s.spv; ph[6] = (uint32_t)s.gin;
}
template <int N>
BB_HD OrigAgent orig_agent(const World<N> &s, int i)
{
    OrigAgent o;
    o.rst = s.rst[i]; o.inb = s.inb[i]; o.allow = s.allow[i];
#pragma unroll
    for (int k = 0; k < 5; k++) o.attr[k] = fbits(s.attr[i][k]);
    o.attr[5] = fbits(s.attr[i][9]);
    return o;
}
template <int N>
BB_HD void capture(Orig<N> &o, const World<N> &s)
{
    game_words(s, o.game);
    phys_words(s, o.phys);
    o.grab[0] = (uint32_t)s.grab; o.grab[1] = (uint32_t)s.holder;
    o.clock = (uint32_t)s.reset_now; o.rng = s.rng_ctr;
#pragma unroll
    for (int i = 0; i < N; i++) o.ag[i] = orig_agent(s, i);
}

template <int NW>
BB_HD bool differ(const uint32_t (&a)[NW], const uint32_t (&b)[NW])
{
    bool d = false;
#pragma unroll
    for (int k = 0; k < NW; k++) d |= a[k] != b[k];
    return d;
}

// The loads of load_world split by owner, for kernels whose N lanes of a
// world load it together (lane i: agent i's columns; lane 0 also the world's).
// Raw words first (load), converted into the world later (commit), so a
// kernel can issue the loads of its next world group early.
struct WorldRaw {  // world-level columns: GameState, WorldClock, RNG counter, ball
    uint32_t g[14], clock, rng, bp[3], bv[3], ph[7], gb[2];
    BB_HD void load(const Params &p, int64_t w)
    {
        const Columns &c = p.c;
        load_words<14>(c.game_state, w, g);
        clock = (uint32_t)c.world_clock[w];
        rng = c.rng_counter[w];
        const uint32_t *b = (const uint32_t *)c.ball_pos + w * 3, *v = (const uint32_t *)c.ball_vel + w * 3;
        const uint32_t *h = (const uint32_t *)c.ball_physics + w * 7;
#pragma unroll
        for (int k = 0; k < 3; k++) { bp[k] = b[k]; bv[k] = v[k]; }
#pragma unroll
        for (int k = 0; k < 7; k++) ph[k] = h[k];
        load_words<2>(c.ball_grabbed, w, gb);
    }
    template <int N>
    BB_HD void commit(World<N> &s) const
    {
        s.g_inb = (int32_t)g[0]; s.g_live = (int32_t)g[1]; s.g_period = bitsf(g[2]); s.g_poss = bitsf(g[3]);
        s.g_h0 = (int32_t)g[4]; s.g_s0 = bitsf(g[5]); s.g_h1 = (int32_t)g[6]; s.g_s1 = bitsf(g[7]);
        s.g_clock = bitsf(g[8]); s.g_shot = bitsf(g[9]); s.g_bask = bitsf(g[10]); s.g_oob = bitsf(g[11]);
        s.g_inbclk = bitsf(g[12]); s.g_1v1 = (int32_t)g[13];
        s.reset_now = (int32_t)clock;
        s.rng_ctr = rng;
        s.bx = bitsf(bp[0]); s.by = bitsf(bp[1]); s.bz = bitsf(bp[2]);
        s.bvx = bitsf(bv[0]); s.bvy = bitsf(bv[1]); s.bvz = bitsf(bv[2]);
        s.fl = (int32_t)ph[0]; s.lta = (int32_t)ph[1]; s.ltt = (int32_t)ph[2]; s.sba = (int32_t)ph[3];
        s.sbt = (int32_t)ph[4]; s.spv = (int32_t)ph[5]; s.gin = (int32_t)ph[6];
        s.grab = (int32_t)gb[0]; s.holder = (int32_t)gb[1];
    }
};

template <int N>
struct AgentRaw {  // agent i's columns (row w*N + i)
    uint32_t a[6], pos[3], ps[3], q[4], v[3], ib[2], at[10], rst, cd, st, t0, t4;
    BB_HD void load(const Params &p, int64_t w, int i)
    {
        const Columns &c = p.c;
        const int64_t r = w * N + i;
        load_words<6>(c.action, r, a);
        load_words<3>(c.agent_pos, r, pos);
        load_words<3>(c.possession, r, ps);
        load_words<4>(c.orientation, r, q);
        load_words<3>(c.agent_vel, r, v);
        load_words<2>(c.inbounding, r, ib);
        load_words<10>(c.attributes, r, at);
        rst = (uint32_t)c.reset[r];
        cd = fbits(c.cooldown[r]);
        st = c.cur_step[r];
        t0 = c.team[r * 5];
        t4 = c.team[r * 5 + 4];
    }
    BB_HD void commit(World<N> &s, int i) const
    {
        s.rst[i] = (int32_t)rst;
#pragma unroll
        for (int k = 0; k < 6; k++) s.act[i][k] = (int32_t)a[k];
        s.px[i] = bitsf(pos[0]); s.py[i] = bitsf(pos[1]); s.pz[i] = bitsf(pos[2]);
        s.has[i] = (int32_t)ps[0]; s.bid[i] = (int32_t)ps[1]; s.pw[i] = (int32_t)ps[2];
        s.qw[i] = bitsf(q[0]); s.qx[i] = bitsf(q[1]); s.qy[i] = bitsf(q[2]); s.qz[i] = bitsf(q[3]);
        s.vx[i] = bitsf(v[0]); s.vy[i] = bitsf(v[1]); s.vz[i] = bitsf(v[2]);
        s.cd[i] = bitsf(cd);
        s.step[i] = st;
        s.inb[i] = (int32_t)ib[0]; s.allow[i] = (int32_t)ib[1];
#pragma unroll
        for (int k = 0; k < 10; k++) s.attr[i][k] = bitsf(at[k]);
        s.team[i] = (int32_t)t0;
        s.dhoop[i] = (int32_t)t4;
        s.rew[i] = 0.f; s.done[i] = 0.f;  // rewritten by tick before any read
#pragma unroll
        for (int k = 0; k < 4; k++) s.msk[i][k] = 0;  // rewritten by actionMaskSystem
    }
};

template <int N>
BB_HD void load_world_shared(World<N> &s, const Params &p, int64_t w)
{
    WorldRaw r;
    r.load(p, w);
    r.commit(s);
}

template <int N>
BB_HD void load_world_agent(World<N> &s, const Params &p, int64_t w, int i)
{
    AgentRaw<N> r;
    r.load(p, w, i);
    r.commit(s, i);
}

// BB_FULL_ROWS: the whole GameState and Attributes rows are rewritten every
// step instead of only their changed words (game/shot clock, Attributes 5-8),
// so a wave's stores cover whole lines of those columns.  A/B (two repeats,
// profiles/r02/o_full_rows_ab.txt): 65 536 x 2 21.85 -> 21.69 us, 262 144 x 2
// 75.5 -> 75.2, N = 4 70.7 -> 69.5, N = 10 323.4 -> 320.6.
#ifndef BB_FULL_ROWS
#define BB_FULL_ROWS 1
#endif

// World-level columns (GameState, WorldClock, RNG counter, ball).  With `o`,
// the event-only words are rewritten only when changed (see Orig).
template <int N, int CA = -1>
BB_HD void store_world_shared(const World<N> &s, const Params &p, int64_t w, const Orig<N> *o = nullptr)
{
    const Columns &c = p.c;
    uint32_t g[14];
    game_words(s, g);
    bool game_ev = o == nullptr || BB_FULL_ROWS;
    if (o) {
#pragma unroll
        for (int k = 0; k < 14; k++)
            if (k != 8 && k != 9) game_ev |= g[k] != o->game[k];
    }
    if (game_ev) {
        store_words<14, CA>(c.game_state, w, g);
    } else {  // game and shot clock only
        const uint32_t clk[2] = {g[8], g[9]};
        store_words<2, CA>(c.game_state + 8, w * 7, clk);  // words 14w+8, 14w+9
    }
    if (!o || (uint32_t)s.reset_now != o->clock) c.world_clock[w] = s.reset_now;
    if (!o || s.rng_ctr != o->rng) c.rng_counter[w] = s.rng_ctr;
    float *bp = c.ball_pos + w * 3, *bv = c.ball_vel + w * 3;
    bp[0] = s.bx; bp[1] = s.by; bp[2] = s.bz;
    bv[0] = s.bvx; bv[1] = s.bvy; bv[2] = s.bvz;
    uint32_t ph[7];
    phys_words(s, ph);
    if (!o || differ(ph, o->phys)) {
        uint32_t *d = (uint32_t *)c.ball_physics + w * 7;
#pragma unroll
        for (int k = 0; k < 7; k++) d[k] = ph[k];
    }
    const uint32_t gb[2] = {(uint32_t)s.grab, (uint32_t)s.holder};
    if (!o || differ(gb, o->grab)) store_words<2, CA>(c.ball_grabbed, w, gb);
}

// Per-agent columns of agent i (row w*N + i of every [W][N][...] column).
// Team changes only inside generate/reset, which write it directly.  With
// `o` (agent i's event-only words as loaded) those are rewritten only when
// changed.  PART: STORE_ALL, or one of the two halves a kernel may store
// from different waves (STORE_ACT_ATTR: Action + Attributes, the columns the
// defence AI and the shot percentage write; STORE_REST: all the others).
enum StorePart : int { STORE_ALL = 0, STORE_ACT_ATTR = 1, STORE_REST = 2 };
template <int N, int CA = -1, int PART = STORE_ALL>
BB_HD void store_world_agent(const World<N> &s, const Params &p, int64_t r, int i, const OrigAgent *o = nullptr)
{
    const Columns &c = p.c;
    constexpr bool AA = PART != STORE_REST, REST = PART != STORE_ACT_ATTR;
    uint32_t a[6], m[4], pos[3], ps[3], q[4], v[3], ib[2], at[10];
#pragma unroll
    for (int k = 0; k < 6; k++) a[k] = (uint32_t)s.act[i][k];
#pragma unroll
    for (int k = 0; k < 4; k++) m[k] = (uint32_t)s.msk[i][k];
    pos[0] = fbits(s.px[i]); pos[1] = fbits(s.py[i]); pos[2] = fbits(s.pz[i]);
    ps[0] = (uint32_t)s.has[i]; ps[1] = (uint32_t)s.bid[i]; ps[2] = (uint32_t)s.pw[i];
    q[0] = fbits(s.qw[i]); q[1] = fbits(s.qx[i]); q[2] = fbits(s.qy[i]); q[3] = fbits(s.qz[i]);
    v[0] = fbits(s.vx[i]); v[1] = fbits(s.vy[i]); v[2] = fbits(s.vz[i]);
    ib[0] = (uint32_t)s.inb[i]; ib[1] = (uint32_t)s.allow[i];
#pragma unroll
    for (int k = 0; k < 10; k++) at[k] = fbits(s.attr[i][k]);
    if (REST) {
        if (!o || s.rst[i] != o->rst) c.reset[r] = s.rst[i];
    }
    if (AA) store_words<6, CA>(c.action, r, a);
    if (REST) {
        store_words<4, CA>(c.action_mask, r, m);
        store_words<3, CA>(c.agent_pos, r, pos);
        c.reward[r] = s.rew[i];
        c.done[r] = s.done[i];
        store_words<3, CA>(c.possession, r, ps);
        store_words<4, CA>(c.orientation, r, q);
        store_words<3, CA>(c.agent_vel, r, v);
        c.cooldown[r] = s.cd[i];
        c.cur_step[r] = s.step[i];
        if (!o || s.inb[i] != o->inb || s.allow[i] != o->allow) store_words<2, CA>(c.inbounding, r, ib);
    }
    if (!AA) return;
    bool attr_ev = o == nullptr || BB_FULL_ROWS;
    if (o) {
#pragma unroll
        for (int k = 0; k < 5; k++) attr_ev |= at[k] != o->attr[k];
        attr_ev |= at[9] != o->attr[5];
    }
    if (attr_ev) {
        store_words<10, CA>(c.attributes, r, at);
    } else {  // target position (5-7) and shot percentage (8)
        uint32_t *d = (uint32_t *)c.attributes + r * 10 + 5;
#pragma unroll
        for (int k = 0; k < 4; k++) d[k] = at[5 + k];
    }
}

template <int N>
BB_HD void store_world(const World<N> &s, const Params &p, int64_t w, const Orig<N> *o = nullptr)
{
    store_world_shared(s, p, w, o);
#pragma unroll
    for (int i = 0; i < N; i++) store_world_agent(s, p, w * N + i, i, o ? &o->ag[i] : nullptr);
}

// Constant columns written once at construction: entity ids, hoop positions.
template <int N>
BB_HD void init_static_columns(const Params &p, int64_t w)
{
#pragma unroll
    for (int i = 0; i < N; i++) p.c.agent_id[w * N + i] = AGENT0_ID + i;
    p.c.ball_id[w] = BALL_ID;
    float *h = p.c.hoop_pos + w * 6;
    h[0] = p.hoop0[0]; h[1] = p.hoop0[1]; h[2] = p.hoop0[2];
    h[3] = p.hoop1[0]; h[4] = p.hoop1[1]; h[5] = p.hoop1[2];
}

// World generation into the columns (obs rows zeroed).
template <int N>
BB_HD void init_world(const Params &p, int64_t w)
{
    World<N> s;
    Ctx c = make_ctx(p, w);
    generate_world(s, c);
    store_world(s, p, w);
    init_static_columns<N>(p, w);
    float *o = p.c.obs + w * N * (int64_t)obs_width(N);
    for (int k = 0; k < N * obs_width(N); k++) o[k] = 0.f;
}

template <int N>
BB_HD void step_one_world(const Params &p, int64_t w)
{
    World<N> s;
    load_world(s, p, w);
    Orig<N> o;
    capture(o, s);
    Ctx c = make_ctx(p, w);
    step_world(s, c);
    store_world(s, p, w, &o);
}

}  // namespace bb
