/*
 * bb_oracle.c -- CPU oracle: plain-C restatement of the reference's per-step
 * task graph.  TEST INFRASTRUCTURE ONLY (see bb_oracle.h for who may use it).
 *
 * Execution model restated: the Madrona CPU TaskGraphExecutor runs, per world,
 * the 19 ParallelFor nodes of src/game.cpp:1463-1526 in graph order; within a
 * node every matching entity is visited in creation order (hoop0, hoop1, ball,
 * agent0..agentN-1 as created by src/gen.cpp:101-206).  Every function below
 * cites the reference lines it restates.  Parity status: partially pinned
 * (bb_oracle.h header; DESIGN.md section "Oracle").
 *
 * Build-defined Madrona details (unpinned, the reference's submodule is absent):
 *   - entity ids: hoop0=0, hoop1=1, ball=2, agent i = 3+i (creation order);
 *   - Vector3::normalize(v) = v * (1.0f / sqrtf(v.length2()));
 *   - RNG: threefry2x32-20; world key = {seed, 0} (every world, as the
 *     reference's shared split_i(initKey(0),0,0)) or {seed, global world};
 *     draw j of a world: U = (tf(worldKey, {j, 0}).x >> 8) * 2^-24.
 */
#define _POSIX_C_SOURCE 199309L
#include "bb_oracle.h"
#include <math.h>
#include <float.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define MAXN 16
#define PH 2147483647 /* ENTITY_ID_PLACEHOLDER, src/constants.hpp:8 */

/* ---------------------------------------------------------------- constants
 * src/constants.hpp:5-99, evaluated in float as the C++ constexprs are. */
static const float K_PI = 3.14159265358979323846f;          /* madrona::math::pi */
static const float K_TS = 1.0f / 62.0f;                     /* constants.hpp:12 */
static const float K_TIME_PER_PERIOD = 10.f;                /* :13 */
static const float K_PPM = 110.f;                           /* :17 */
static const float K_HOOP_ZONE = 0.1f;                      /* :24 */
static const float K_AGENT_SIZE = 0.2f;                     /* :39 */
static const float K_SHOULDER = (float)0.4290;              /* :40 (double literal) */
static const float K_DEPTH = (float).1;                     /* :41 */
static const float K_GUARD = .2f;                           /* :45 */
static const float K_START_STD = 5.f;                       /* :46 */
static const float K_DEFAULT_SPEED = 3.f;                   /* :47 */
static const float K_DEF_SLOW = 0.2f;                       /* :48 */
static const float K_DEF_REACT = 10.f;                      /* :49 */
static const float K_SPAWN_R = 8.f;                         /* :50 */
static const float K_BALL_SLOW = 0.9f;                      /* :55 */
static const float K_DIST_DEV = .008f, K_DEF_DEV = .002f, K_VEL_DEV = .001f; /* :59-61 */
static const float K_COURT_L = 28.65f, K_COURT_W = 15.24f;  /* :67-68 */
static const float K_MARGIN = 1.1f;                         /* :71 */
static const float K_HOOP_FROM_BASE = 1.575f;               /* :84 */
static const float K_ARC = 7.24f, K_CORNER_SIDE = 0.91f, K_CORNER_LEN = 4.27f; /* :91-93 */

static float g_world_w, g_world_h, g_cminx, g_cmaxx, g_cminy, g_cmaxy;
static void init_court(void)
{
    volatile float l = K_COURT_L, w = K_COURT_W, m = K_MARGIN;
    g_world_w = l * m;                     /* :72 */
    g_world_h = w * m;                     /* :73 */
    g_cminx = (g_world_w - l) / 2.0f;      /* :76 */
    g_cmaxx = g_cminx + l;                 /* :77 */
    g_cminy = (g_world_h - w) / 2.0f;      /* :78 */
    g_cmaxy = g_cminy + w;                 /* :79 */
}

/* ---------------------------------------------------------------- math mode */
static int g_math = OR_MATH_CR;
static float m_sinf(float x) { return g_math != OR_MATH_CR ? sinf(x) : (float)sin((double)x); }
static float m_cosf(float x) { return g_math != OR_MATH_CR ? cosf(x) : (float)cos((double)x); }
static float m_atan2f(float y, float x) { return g_math != OR_MATH_CR ? atan2f(y, x) : (float)atan2((double)y, (double)x); }
static float m_atanf(float x) { return g_math != OR_MATH_CR ? atanf(x) : (float)atan((double)x); }
static float m_acosf(float x) { return g_math != OR_MATH_CR ? acosf(x) : (float)acos((double)x); }
/* The unqualified erf / acos / exp of game.cpp:746,808,868 on float arguments:
 * the double overloads (C's ::erf etc., promoted argument) unless the build's
 * headers put the float overloads into the global namespace.
 * OR_MATH_LIBM_FLOAT binds them to erff / acosf / expf, to measure how far a
 * reference built that way would diverge; every other mode takes the double
 * reading, as the product does. */
static float u_erf(float x) { return g_math == OR_MATH_LIBM_FLOAT ? erff(x) : (float)erf((double)x); }
static float u_acos(float x) { return g_math == OR_MATH_LIBM_FLOAT ? acosf(x) : (float)acos((double)x); }
static float u_exp_add(float r, float x)
{
    return g_math == OR_MATH_LIBM_FLOAT ? r + expf(x) : (float)((double)r + exp((double)x));
}

/* ---------------------------------------------------------------- vectors
 * madrona::math Vector3 / Quat semantics (operator order as written in the
 * reference; rotateVec pinned by scripts/viewer.py:59-65). */
typedef struct { float x, y, z; } V3;
typedef struct { float w, x, y, z; } Q4;
static V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
static V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static V3 vmul(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static float vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static float vlen2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static float vlen(V3 a) { return sqrtf(vlen2(a)); }
static V3 vnorm(V3 a) { return vmul(a, 1.0f / sqrtf(vlen2(a))); }
static V3 vcross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static float clampf_(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
static Q4 qaxis(float angle, V3 n)
{
    float c = m_cosf(0.5f * angle), s = m_sinf(0.5f * angle);
    Q4 q; q.w = c; q.x = s * n.x; q.y = s * n.y; q.z = s * n.z; return q;
}
static Q4 qmul(Q4 a, Q4 b)
{
    Q4 r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x;
    r.z = a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w;
    return r;
}
static V3 qrot(Q4 q, V3 v)
{
    V3 p = v3(q.x, q.y, q.z);
    V3 pv = vcross(p, v);
    V3 ppv = vcross(p, pv);
    return vadd(v, vmul(vadd(vmul(pv, q.w), ppv), 2.f));
}
static const V3 FWD = {0.f, 1.f, 0.f}; /* AGENT_BASE_FORWARD, constants.hpp:54 */

/* ---------------------------------------------------------------- RNG */
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
void oracle_threefry2x32(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t out[2])
{
    /* Random123 threefry2x32, 20 rounds (Salmon et al., SC'11). */
    static const int R[8] = {13, 15, 26, 6, 17, 29, 16, 24};
    uint32_t ks[3] = {k0, k1, 0x1BD11BDAu ^ k0 ^ k1};
    uint32_t x0 = c0 + ks[0], x1 = c1 + ks[1];
    for (int r = 0; r < 20; r++) {
        x0 += x1; x1 = rotl32(x1, R[r % 8]); x1 ^= x0;
        if ((r & 3) == 3) {
            uint32_t s = (uint32_t)((r + 1) >> 2);
            x0 += ks[s % 3]; x1 += ks[(s + 1) % 3] + s;
        }
    }
    out[0] = x0; out[1] = x1;
}

/* ---------------------------------------------------------------- world */
typedef struct {
    int32_t id;
    int32_t reset;                  /* Reset */
    int32_t act[6];                 /* Action: move, moveAngle, rotate, grab, pass, shoot */
    int32_t mask[4];                /* ActionMask: can_move, can_grab, can_pass, can_shoot */
    float cooldown;                 /* GrabCooldown */
    V3 pos;                         /* Position */
    float reward, done;             /* Reward, Done */
    uint32_t cur_step;              /* CurStep */
    int32_t has_ball, ball_id, points_worth; /* InPossession */
    Q4 q;                           /* Orientation */
    int32_t im_inb, allowed_move;   /* Inbounding */
    int32_t team; V3 color; int32_t def_hoop; /* Team */
    float st_points, st_fouls;      /* Stats */
    float max_speed, quickness, shooting, ft, reaction; V3 target; float shot_pct; /* Attributes */
    V3 vel;                         /* Velocity */
} OAgent;

typedef struct {
    int32_t id; V3 pos; V3 vel;
    int32_t in_flight, last_agent, last_team, shot_agent, shot_team, shot_value, going_in; /* BallPhysics */
    int32_t grabbed, holder;        /* Grabbed */
} OBall;

typedef struct { int32_t id; V3 pos; float radius; V3 center; } OHoop;

typedef struct {
    int32_t inbounding, live; float period, poss; int32_t h0; float s0; int32_t h1; float s1;
    float clock, shot, baskets, oob, inb_clock; int32_t one_v_one;
} OGame;

typedef struct {
    OGame gs;
    int32_t reset_now;              /* WorldClock singleton */
    uint32_t key0, key1, ctr;       /* Sim::rng */
    OAgent ag[MAXN];
    OBall ball;
    OHoop hoop[2];
    float *obs;                     /* [N][obs_w] */
} OWorld;

typedef struct {
    oracle_cfg cfg;
    int n, obs_w;
    float width, height;
    uint32_t flags;
    OWorld *w;
    float *obs_store;
    int64_t ev[OR_NUM_EVENTS];      /* cumulative event counts (test coverage) */
} Oracle;

static Oracle *G; /* current oracle (single-threaded checker) */
#define EV(k) (G->ev[(k)]++)

static float sample_uniform(OWorld *w, float lo, float hi) /* helper.cpp:8-11 */
{
    uint32_t o[2];
    oracle_threefry2x32(w->key0, w->key1, w->ctr, 0u, o);
    w->ctr++;
    float u = (float)(o[0] >> 8) * (1.0f / 16777216.0f);
    return lo + (hi - lo) * u;
}

static V3 vec_to_center(V3 p) /* helper.cpp:44-48 */
{
    return vnorm(vsub(v3(G->cfg.start_x, G->cfg.start_y, 0.f), p));
}

static Q4 rot_between(V3 a, V3 b) /* helper.cpp:14-42 */
{
    a = vnorm(a); b = vnorm(b);
    float d = vdot(a, b);
    if (d > 0.999999f) { Q4 id = {1.f, 0.f, 0.f, 0.f}; return id; }
    if (d < -0.999999f) return qaxis(K_PI, v3(0.f, 0.f, 1.f));
    V3 ax = vnorm(vcross(a, b));
    return qaxis(m_acosf(d), ax);
}

static int32_t shot_value(V3 p, V3 hz) /* helper.cpp:50-81 */
{
    float d = vlen(vsub(p, hz));
    int corner = (p.y < g_cminy + K_CORNER_SIDE) || (p.y > g_cminy + K_COURT_W - K_CORNER_SIDE);
    if (corner) {
        if (hz.x < g_world_w / 2.0f) { if (p.x <= g_cminx + K_CORNER_LEN) return 3; }
        else { if (p.x >= g_cminx + K_COURT_L - K_CORNER_LEN) return 3; }
    }
    if (d >= K_ARC) return 3;
    return 2;
}

static void setup_positions(OWorld *w, int32_t *off_id, V3 *ball_at) /* helper.cpp:108-160 */
{
    const int n = G->n;
    for (int i = 0; i < n; i++) {
        OAgent *a = &w->ag[i];
        if (w->gs.one_v_one == 1) {
            if (i == 0) {
                V3 base = v3(G->cfg.start_x + ((float)i * 2.f), G->cfg.start_y, 0.f);
                float xd = sample_uniform(w, -K_START_STD, K_START_STD);
                float yd = sample_uniform(w, -K_START_STD, K_START_STD);
                a->pos = vadd(base, v3(xd, yd, 0.f));
                a->pos.x = clampf_(a->pos.x, 0.f, G->width);
                a->pos.y = clampf_(a->pos.y, 0.f, G->height);
                *ball_at = a->pos;
                *off_id = a->id;
                a->has_ball = 1; a->ball_id = w->ball.id; a->points_worth = 2;
            } else {
                float ang = sample_uniform(w, 0.f, 2.f * K_PI);
                V3 off = v3(K_SPAWN_R * m_cosf(ang), K_SPAWN_R * m_sinf(ang), 0.f);
                a->pos = vadd(*ball_at, off);
                a->pos.x = clampf_(a->pos.x, 0.f, G->width);
                a->pos.y = clampf_(a->pos.y, 0.f, G->height);
                a->has_ball = 0; a->ball_id = PH; a->points_worth = 2;
            }
        } else {
            a->pos = v3((G->cfg.start_x - 1.f) - (float)(-2 * (i % 2)),
                        (G->cfg.start_y - 2.f) + (float)(i / 2), 0.f);
            if (i == 0) { *off_id = a->id; a->has_ball = 1; a->ball_id = w->ball.id; a->points_worth = 2; }
            else { a->has_ball = 0; a->ball_id = PH; a->points_worth = 2; }
        }
        a->max_speed = K_DEFAULT_SPEED - (float)i * K_DEF_SLOW;
        a->quickness = 1.f; a->shooting = 0.f; a->ft = 0.f;
        a->reaction = (float)i * K_DEF_REACT;
        a->target = a->pos; a->shot_pct = 0.f;
    }
}

static Q4 start_orientation(int i) /* gen.cpp:196, 277 */
{
    return (i % 2 == 0) ? qaxis(-K_PI / 2.0f, v3(0.f, 0.f, 1.f)) : qaxis(K_PI / 2.0f, v3(0.f, 0.f, 1.f));
}

static void generate_world(OWorld *w, int64_t global_index) /* gen.cpp:13-214 + sim.cpp:86-96 */
{
    const int n = G->n;
    memset(&w->gs, 0, sizeof(w->gs));
    w->gs.inbounding = 0; w->gs.live = 1; w->gs.period = 1.f; w->gs.poss = 0.f;
    w->gs.h0 = 0; w->gs.s0 = 0.f; w->gs.h1 = 1; w->gs.s1 = 0.f;
    w->gs.clock = K_TIME_PER_PERIOD; w->gs.shot = 24.f; w->gs.baskets = 0.f; w->gs.oob = 0.f;
    w->gs.inb_clock = 0.f; w->gs.one_v_one = (G->flags & OR_FLAG_FULL_GAME) ? 0 : 1;
    w->reset_now = 0;
    /* Sim::Sim: rng = split_i(initKey(seed), 0, 0) for every world; build
     * definition: key {seed, 0} (or {seed, global world index}). */
    w->key0 = G->cfg.seed;
    w->key1 = (G->flags & OR_FLAG_PER_WORLD_RNG) ? (uint32_t)global_index : 0u;
    w->ctr = 0;
    float csx = (G->width - K_COURT_L) / 2.0f;
    float ccy = G->height / 2.0f;
    w->hoop[0].id = 0; w->gs.h0 = 0;
    w->hoop[0].pos = v3(csx + K_HOOP_FROM_BASE, ccy, 0.f);
    w->hoop[0].radius = K_HOOP_ZONE; w->hoop[0].center = w->hoop[0].pos;
    w->hoop[1].id = 1; w->gs.h1 = 1;
    w->hoop[1].pos = v3(csx + K_COURT_L - K_HOOP_FROM_BASE, ccy, 0.f);
    w->hoop[1].radius = K_HOOP_ZONE; w->hoop[1].center = w->hoop[1].pos;

    OBall *b = &w->ball;
    b->id = 2;
    b->pos = v3(G->cfg.start_x, G->cfg.start_y, 0.f);
    b->grabbed = 0; b->holder = PH;
    b->in_flight = 0; b->last_agent = PH; b->last_team = PH; b->shot_agent = PH; b->shot_team = PH;
    b->shot_value = 2; b->going_in = 0;
    b->vel = v3(0.f, 0.f, 0.f);

    int32_t off_id = PH;
    V3 ball_at = v3(G->cfg.start_x, G->cfg.start_y, 0.f);
    for (int i = 0; i < n; i++) {
        OAgent *a = &w->ag[i];
        memset(a, 0, sizeof(*a));
        a->id = 3 + i;
        a->im_inb = 0; a->allowed_move = 1;
        a->q = start_orientation(i);
        a->team = i % 2;
        a->color = (i % 2 == 0) ? v3(0.f, 100.f, 255.f) : v3(128.f, 0.f, 128.f);
        a->def_hoop = (i % 2 == 0) ? w->gs.h0 : w->gs.h1;
    }
    setup_positions(w, &off_id, &ball_at);
    if (w->gs.one_v_one == 1) { b->grabbed = 1; b->holder = off_id; }
}

static void reset_world(OWorld *w) /* gen.cpp:216-316 */
{
    const int n = G->n;
    OGame *g = &w->gs;
    if (g->clock <= 0.f && (float)g->one_v_one == 0.f) {
        if (g->period < 4.f || g->s0 == g->s1) {
            g->period += 1.f; g->clock = K_TIME_PER_PERIOD; g->shot = 24.f; g->live = 1; g->inbounding = 0;
            EV(OR_EV_PERIOD_ADVANCE);
        } else {
            g->live = 0;
            EV(OR_EV_GAME_END);
        }
    } else {
        int32_t h0 = g->h0, h1 = g->h1, ovo = g->one_v_one;
        g->inbounding = 0; g->live = 1; g->period = 1.f; g->poss = 0.f; g->h0 = h0; g->s0 = 0.f;
        g->h1 = h1; g->s1 = 0.f; g->clock = K_TIME_PER_PERIOD; g->shot = 24.f; g->baskets = 0.f;
        g->oob = 0.f; g->inb_clock = 0.f; g->one_v_one = ovo;
    }
    const V3 colors[2] = {{0.f, 100.f, 255.f}, {255.f, 0.f, 100.f}};
    int32_t off_id = PH;
    V3 ball_at = v3(G->cfg.start_x, G->cfg.start_y, 0.f);
    for (int i = 0; i < n; i++) {
        OAgent *a = &w->ag[i];
        memset(a->act, 0, sizeof(a->act));
        memset(a->mask, 0, sizeof(a->mask));
        a->reset = 0; a->im_inb = 0; a->allowed_move = 1; a->done = 1.f; a->cur_step = 0;
        a->q = start_orientation(i);
        a->cooldown = 0.f; a->st_points = 0.f; a->st_fouls = 0.f; a->vel = v3(0.f, 0.f, 0.f);
        a->team = i % 2; a->color = colors[i % 2];
        a->def_hoop = (i % 2 == 0) ? g->h0 : g->h1;
    }
    setup_positions(w, &off_id, &ball_at);
    OBall *b = &w->ball;
    b->pos = ball_at;
    b->in_flight = 0; b->last_agent = PH; b->last_team = PH; b->shot_agent = PH; b->shot_team = PH;
    b->shot_value = 2; b->going_in = 0;
    b->vel = v3(0.f, 0.f, 0.f);
    if (g->one_v_one == 1) { b->grabbed = 1; b->holder = off_id; }
    else { b->grabbed = 0; b->holder = PH; }
}

static void assign_inbounder(OWorld *w, V3 ball_pos, int32_t team, Q4 orient, int is_oob) /* game.cpp:14-53 */
{
    float assigned = 0.0f;
    for (int i = 0; i < G->n; i++) {
        OAgent *a = &w->ag[i];
        if (a->team == team && assigned == 0.f) {
            assigned = 1.f;
            a->im_inb = 1;
            a->pos = ball_pos;
            w->ball.grabbed = 1; w->ball.holder = a->id;
            a->has_ball = 1; a->ball_id = w->ball.id;
            a->q = orient;
        }
    }
    if (assigned > 0.f) {
        w->gs.poss = (float)team;
        w->gs.inbounding = 1;
        w->gs.inb_clock = 5.f;
        if (is_oob) w->gs.oob += 1.f;
        EV(OR_EV_INBOUND_START);
    }
}

/* ------------------------------------------------------------------ systems */
static void sys_tick(OWorld *w, OAgent *a) /* game.cpp:969-988 */
{
    (void)w;
    a->reward = 0.f;
    if (a->reset == 1) { a->done = 1.f; a->cur_step = 0; }
    else { a->done = 0.f; a->cur_step++; }
    a->cooldown = fmaxf(0.f, a->cooldown - 1.f);
}

static void sys_action_mask(OWorld *w, OAgent *a) /* game.cpp:489-533 */
{
    a->mask[0] = 1; a->mask[1] = 1; a->mask[2] = 0; a->mask[3] = 0;
    if (a->has_ball == 1) { a->mask[2] = 1; a->mask[3] = 1; }
    if (w->gs.inbounding == 1) {
        a->mask[3] = 0; a->mask[1] = 0;
        if (a->im_inb == 1 && w->gs.live == 0) a->mask[0] = 0;
    }
    if (a->cooldown > 0.f) a->mask[1] = 0;
    if (!(G->flags & OR_FLAG_NO_TAG_MASK)) { a->mask[2] = 0; a->mask[1] = 0; }
}

static void sys_move_agent(OWorld *w, OAgent *a) /* game.cpp:410-486 */
{
    (void)w;
    if (a->act[2] != 0) {
        float turn = (a->act[2] == 1) ? (K_PI / 180.f) * 6.f : (K_PI / 180.f) * -6.f;
        a->q = qmul(qaxis(turn, v3(0.f, 0.f, 1.f)), a->q);
    }
    if (a->mask[0] == 0) return;
    float ang = (float)a->act[1] * (K_PI / 4.0f);
    V3 dv = vmul(vmul(v3(m_sinf(ang), -m_cosf(ang), 0.f), a->quickness), (float)a->act[0]);
    float maxs = a->max_speed;
    V3 f = qrot(a->q, FWD);
    float d = 0.f;
    if (vlen2(a->vel) > 1e-6f) d = vdot(vnorm(a->vel), f);
    if (d < -0.1f) { maxs *= .1f; dv = vmul(dv, .1f); }
    else if (d <= 0.8f) { maxs *= .7f; dv = vmul(dv, .1f); }
    a->vel = vadd(a->vel, dv);
    if (a->has_ball == 1) maxs *= K_BALL_SLOW;
    if (vlen(a->vel) > maxs) a->vel = vmul(a->vel, maxs / vlen(a->vel));
    float dx = a->vel.x * K_TS, dy = a->vel.y * K_TS;
    float nx = clampf_(a->pos.x + dx, 0.f, G->width);
    float ny = clampf_(a->pos.y + dy, 0.f, G->height);
    /* Grid wall lookup (game.cpp:472-484): the binding builds an all-empty
     * grid (bindings.cpp:7-11), so the move is always accepted. */
    a->pos.x = nx; a->pos.y = ny;
    a->vel = vmul(a->vel, .95f);
}

static void sys_grab(OWorld *w, OAgent *a) /* game.cpp:164-239 */
{
    if (a->mask[1] == 0 || a->act[3] == 0) return;
    a->cooldown = 10.f;
    a->act[3] = 0;
    OBall *b = &w->ball;
    if (b->in_flight == 1) return;
    int holding = (a->has_ball == 1 && b->grabbed == 1 && b->holder == a->id);
    if (holding) {
        a->ball_id = PH; a->has_ball = 0; b->holder = PH; b->grabbed = 0;
        return;
    }
    float d = vlen(vsub(b->pos, a->pos));
    if (d <= 0.3f) {
        if ((float)w->gs.one_v_one == 1.f && (float)a->team != w->gs.poss) {
            EV(OR_EV_DEFENDER_GRAB_RESET);
            w->reset_now = 1;
            return;
        }
        for (int j = 0; j < G->n; j++) {
            OAgent *o = &w->ag[j];
            if (o->ball_id == b->id) { o->has_ball = 0; o->ball_id = PH; o->cooldown = 62.0f; }
        }
        EV(OR_EV_GRAB);
        a->has_ball = 1; a->ball_id = b->id;
        b->holder = a->id; b->grabbed = 1; b->in_flight = 0;
        b->vel = v3(0.f, 0.f, 0.f);
        b->shot_agent = PH; b->shot_team = PH; b->shot_value = 2;
        w->gs.poss = (float)a->team;
        w->gs.live = 1;
    }
}

static void sys_pass(OWorld *w, OAgent *a) /* game.cpp:243-270 */
{
    if (a->mask[2] == 0 || a->act[4] == 0) return;
    OBall *b = &w->ball;
    if (b->holder == a->id) {
        EV(OR_EV_PASS);
        b->grabbed = 0; b->holder = PH;
        a->has_ball = 0; a->ball_id = PH; a->im_inb = 0;
        b->vel = qrot(a->q, v3(0.f, 0.1f, 0.f));
        w->gs.inbounding = 0;
    }
}

static void sys_shoot(OWorld *w, OAgent *a) /* game.cpp:273-407 */
{
    if (a->mask[3] == 0 || a->act[5] == 0) return;
    V3 pos = a->pos; /* by-value Position parameter */
    V3 target = v3(0.f, 0.f, 0.f);
    float radius = 0.f;
    for (int h = 0; h < 2; h++)
        if (w->hoop[h].id != a->def_hoop) { target = w->hoop[h].center; radius = w->hoop[h].radius; }
    V3 ideal = vsub(target, pos);
    float intended = m_atan2f(ideal.x, ideal.y);
    float dist = vlen(ideal);
    float dstd = K_DIST_DEV * dist;
    float dev_d = sample_uniform(w, -dstd, dstd);
    float dev_def = 0.0f;
    float nd = INFINITY;
    for (int j = 0; j < G->n; j++) {
        OAgent *o = &w->ag[j];
        if (o->team != a->team) {
            float dd = vlen(vsub(pos, o->pos));
            if (dd < nd) nd = dd;
        }
    }
    if (nd < 2.0f) {
        float s = K_DEF_DEV / (nd + 0.1f);
        dev_def = sample_uniform(w, -s, s);
    }
    float dev_v = 0.0f;
    if (a->act[0] > 0) {
        float s = K_VEL_DEV * vlen(a->vel);
        dev_v = sample_uniform(w, -s, s);
    }
    float total = dev_d + dev_def + dev_v;
    float dir = intended + total;
    V3 fs = v3(m_sinf(dir), m_cosf(dir), 0.f);
    float going = 0.0f;
    float along = vdot(ideal, fs);
    if (along < 0.f) going = 0.0f;
    else {
        float cd2 = vlen2(ideal) - along * along;
        going = (cd2 <= radius * radius) ? 1.0f : 0.0f;
    }
    a->q = rot_between(FWD, fs);
    OBall *b = &w->ball;
    if (b->holder == a->id) {
        int32_t spv = shot_value(pos, target);
        EV(OR_EV_SHOT);
        if (going == 1.f) { b->going_in = 1; w->gs.baskets += 1.f; EV(OR_EV_SHOT_GOING_IN); }
        else a->reward -= 1.f;
        b->grabbed = 0; b->holder = PH;
        a->has_ball = 0; a->ball_id = PH; a->im_inb = 0;
        b->vel = vmul(fs, .1f);
        b->in_flight = 1;
        b->shot_agent = a->id; b->shot_team = a->team; b->shot_value = spv;
        b->last_agent = a->id; b->last_team = a->team;
    }
}

static void sys_move_ball(OWorld *w) /* game.cpp:82-125 */
{
    OBall *b = &w->ball;
    for (int i = 0; i < G->n; i++) {
        OAgent *a = &w->ag[i];
        if (a->has_ball == 1 && b->grabbed == 1 && b->holder == a->id) b->pos = a->pos;
    }
    if (vlen(b->vel) == 0.f || b->grabbed == 1) return;
    float nx = clampf_(b->pos.x + b->vel.x, 0.f, G->width);
    float ny = clampf_(b->pos.y + b->vel.y, 0.f, G->height);
    float nz = b->pos.z + b->vel.z;
    b->pos = v3(nx, ny, nz); /* empty grid: never a wall (game.cpp:118-124) */
}

static void sys_shot_pct(OWorld *w, OAgent *a) /* game.cpp:758-809 */
{
    if (a->has_ball == 0) { a->shot_pct = 0.f; return; }
    V3 hoop = (w->hoop[0].id != a->def_hoop) ? w->hoop[0].pos : w->hoop[1].pos;
    float dh = vlen(vsub(hoop, a->pos));
    float nd = INFINITY;
    for (int j = 0; j < G->n; j++) {
        OAgent *o = &w->ag[j];
        if (o->team != a->team) {
            float dd = vlen(vsub(a->pos, o->pos));
            if (dd < nd) nd = dd;
        }
    }
    float dstd = K_DIST_DEV * dh;
    float defstd = K_DEF_DEV / nd + .0001f;
    float vstd = K_VEL_DEV * vlen(a->vel);
    float fstd = sqrtf((dstd * dstd / 3.f) + (defstd * defstd / 3.f) + (vstd * vstd / 3.f));
    float mma = m_atanf(K_HOOP_ZONE / dh);
    float z = mma / fstd;
    a->shot_pct = u_erf(z / sqrtf(2.f));
}

static void sys_score(OWorld *w, OHoop *h) /* game.cpp:873-953 */
{
    OBall *b = &w->ball;
    OGame *g = &w->gs;
    float dx = b->pos.x - h->pos.x, dy = b->pos.y - h->pos.y;
    float d = sqrtf(dx * dx + dy * dy);
    if (d <= h->radius && (float)b->in_flight == 1.f) {
        int32_t pts = b->shot_value;
        int32_t inb_team = 0;
        EV(OR_EV_MAKE);
        for (int j = 0; j < G->n; j++) {
            OAgent *a = &w->ag[j];
            if (a->def_hoop == h->id) inb_team = a->team;
            if (a->id == b->shot_agent)
                a->st_points += (float)((a->def_hoop == h->id) ? -b->shot_value : b->shot_value);
        }
        V3 spot;
        if (h->id == g->h0) {
            g->s1 += (float)pts;
            spot = v3(g_cminx, h->pos.y + (K_PPM / 60.f), 0.f);
        } else {
            g->s0 += (float)pts;
            spot = v3(g_cmaxx, h->pos.y + (K_PPM / 60.f), 0.f);
        }
        g->baskets += 1.f;
        b->in_flight = 0;
        b->vel = v3(0.f, 0.f, 0.f);
        b->shot_agent = PH; b->shot_team = PH; b->shot_value = 2; b->going_in = 0;
        if ((float)g->one_v_one == 0.f) {
            b->pos = spot;
            Q4 o = rot_between(FWD, vec_to_center(b->pos));
            assign_inbounder(w, spot, inb_team, o, 0);
        } else {
            w->reset_now = 1;
        }
    }
}

static int offense_agent_index(OWorld *w) /* game.cpp:1012-1018, 1072-1078 */
{
    int off = 0;
    for (int i = 1; i < G->n; i++)
        if ((float)w->ag[i].team == w->gs.poss) off = i;
    return off;
}

static void sys_out_of_bounds(OWorld *w) /* game.cpp:1055-1113 */
{
    OBall *b = &w->ball;
    OGame *g = &w->gs;
    if ((b->pos.x < g_cminx || b->pos.x > g_cmaxx || b->pos.y < g_cminy || b->pos.y > g_cmaxy) &&
        (float)g->inbounding == 0.f) {
        if ((float)g->one_v_one == 1.f) {
            w->ag[offense_agent_index(w)].reward -= 100.f;
            w->reset_now = 1;
            EV(OR_EV_OOB_1V1);
        } else {
            b->in_flight = 0;
            b->vel = v3(0.f, 0.f, 0.f);
            g->live = 0;
            EV(OR_EV_OOB_TURNOVER);
            int32_t new_team = 1 - b->last_team;
            for (int i = 0; i < G->n; i++) {
                OAgent *a = &w->ag[i];
                if (a->has_ball == 1 && a->ball_id == b->id) {
                    a->pos = vadd(a->pos, vec_to_center(a->pos));
                    a->has_ball = 0; a->ball_id = PH;
                }
            }
            Q4 o = rot_between(FWD, vec_to_center(b->pos));
            assign_inbounder(w, b->pos, new_team, o, 1);
        }
    }
}

static void sys_last_touch(OWorld *w) /* game.cpp:1034-1051 */
{
    OBall *b = &w->ball;
    for (int i = 0; i < G->n; i++) {
        OAgent *a = &w->ag[i];
        float d = vlen(vsub(b->pos, a->pos));
        if (d <= K_AGENT_SIZE) { b->last_agent = a->id; b->last_team = a->team; }
    }
}

static void sys_clock(OWorld *w) /* game.cpp:992-1030 */
{
    OGame *g = &w->gs;
    if ((float)g->live > 0.5f && g->clock > 0.f) { g->clock -= K_TS; g->shot -= K_TS; }
    if ((float)g->inbounding > 0.5f) g->inb_clock -= K_TS;
    if (g->clock <= 0.f && (float)g->live > 0.5f) {
        w->ag[offense_agent_index(w)].reward += 10.f;
        w->reset_now = 1;
        EV(OR_EV_CLOCK_EXPIRY);
    }
    if (g->shot < 0.f) g->shot = 0.f;
}

static void sys_inbound_violation(OWorld *w) /* game.cpp:1116-1157 */
{
    OGame *g = &w->gs;
    if (!((float)g->inbounding > 0.5f && g->inb_clock <= 0.f)) return;
    int32_t cur = (int32_t)g->poss;
    int32_t new_team = 1 - cur;
    int32_t turn_id = PH;
    g->live = 0;
    EV(OR_EV_INBOUND_VIOLATION);
    for (int i = 0; i < G->n; i++) {
        OAgent *a = &w->ag[i];
        if ((float)a->im_inb > 0.5f) {
            turn_id = a->ball_id;
            a->im_inb = 0; a->has_ball = 0; a->ball_id = PH;
            a->pos = vadd(a->pos, vec_to_center(a->pos));
        }
    }
    if (turn_id != PH) {
        OBall *b = &w->ball;
        if (b->id == turn_id) {
            b->grabbed = 0; b->holder = PH;
            Q4 o = rot_between(FWD, vec_to_center(b->pos));
            assign_inbounder(w, b->pos, new_team, o, 1);
        }
    }
}

static void sys_reset(OWorld *w) /* game.cpp:957-967 */
{
    if (w->reset_now == 0) return;
    EV(OR_EV_WORLD_RESET);
    reset_world(w);
    w->reset_now = 0;
}

static void sys_points_worth(OWorld *w, OAgent *a) /* game.cpp:129-161 */
{
    V3 target = v3(0.f, 0.f, 0.f);
    int found = 0;
    for (int h = 0; h < 2; h++)
        if (w->hoop[h].id != a->def_hoop) { target = w->hoop[h].center; found = 1; break; }
    a->points_worth = found ? shot_value(a->pos, target) : 2;
}

typedef struct { float mn, mx; } Proj;
static Proj project_rect(const V3 *v, V3 axis) /* helper.cpp:85-100 */
{
    Proj p; p.mn = vdot(v[0], axis); p.mx = p.mn;
    for (int i = 1; i < 4; i++) {
        float d = vdot(v[i], axis);
        if (d < p.mn) p.mn = d;
        if (d > p.mx) p.mx = d;
    }
    return p;
}

static void sys_collision(OWorld *w, OAgent *a) /* game.cpp:537-648 */
{
    for (int i = 0; i < G->n; i++) {
        OAgent *bb = &w->ag[i];
        if (a->id >= bb->id) continue;
        V3 ca = a->pos;
        V3 fa = qrot(a->q, FWD);
        V3 ra = v3(fa.y, -fa.x, 0.f);
        V3 hwa = vmul(ra, K_SHOULDER / 2.0f), hda = vmul(fa, K_DEPTH / 2.0f);
        V3 va[4] = {vadd(vsub(ca, hda), hwa), vsub(vsub(ca, hda), hwa), vsub(vadd(ca, hda), hwa), vadd(vadd(ca, hda), hwa)};
        V3 cb = bb->pos;
        V3 fb = qrot(bb->q, FWD);
        V3 rb = v3(fb.y, -fb.x, 0.f);
        V3 hwb = vmul(rb, K_SHOULDER / 2.0f), hdb = vmul(fb, K_DEPTH / 2.0f);
        V3 vb[4] = {vadd(vsub(cb, hdb), hwb), vsub(vsub(cb, hdb), hwb), vsub(vadd(cb, hdb), hwb), vadd(vadd(cb, hdb), hwb)};
        V3 axes[4] = {vnorm(ra), vnorm(fa), vnorm(rb), vnorm(fb)};
        int colliding = 1;
        float min_ov = FLT_MAX;
        V3 mtv = v3(0.f, 0.f, 0.f);
        for (int j = 0; j < 4; j++) {
            Proj pa = project_rect(va, axes[j]), pb = project_rect(vb, axes[j]);
            if (!(pa.mx > pb.mn && pb.mx > pa.mn)) { colliding = 0; break; }
            float ov = fminf(pa.mx, pb.mx) - fmaxf(pa.mn, pb.mn);
            if (ov < min_ov) { min_ov = ov; mtv = axes[j]; }
        }
        if (colliding) {
            EV(OR_EV_CONTACT);
            if (w->gs.poss == (float)a->team) {
                EV(OR_EV_TAG);
                a->reward -= 10.f;
                bb->reward += 10.f;
                w->reset_now = 1;
            }
            V3 corr = mtv;
            if (vdot(vsub(cb, ca), corr) < 0.f) corr = vneg(corr);
            a->pos = vsub(a->pos, vmul(vmul(corr, min_ov), 0.5f));
            bb->pos = vadd(bb->pos, vmul(vmul(corr, min_ov), 0.5f));
        }
    }
}

static void sys_defense(OWorld *w, OAgent *a) /* game.cpp:651-755 */
{
    if (w->gs.poss == (float)a->team) { a->act[0] = 0; return; }
    a->act[3] = 1;
    V3 guard = v3(0.f, 0.f, 0.f);
    int found = 0;
    for (int i = 0; i < G->n; i++) {
        OAgent *o = &w->ag[i];
        if (o->has_ball == 1 && found == 0) {
            for (int h = 0; h < 2; h++) {
                if (a->def_hoop == w->hoop[h].id) {
                    V3 hd = vsub(w->hoop[h].pos, o->pos);
                    if (vlen2(hd) > 1e-6f) guard = vadd(o->pos, vmul(vnorm(hd), K_GUARD));
                    else guard = o->pos;
                    found = 1;
                }
            }
        }
    }
    if (found == 0) { a->act[0] = 0; return; }
    V3 cur = a->target;
    float f = a->reaction * K_TS;
    a->target = vadd(cur, vmul(vsub(guard, cur), f));
    V3 mv = vsub(a->target, a->pos);
    if (vlen2(mv) < 0.01f) { a->act[0] = 0; return; }
    static const float dirs[8][2] = {{0.f, -1.f}, {1.f, -1.f}, {1.f, 0.f}, {1.f, 1.f},
                                     {0.f, 1.f}, {-1.f, 1.f}, {-1.f, 0.f}, {-1.f, -1.f}};
    V3 desired = vnorm(mv);
    float maxd = -2.f;
    int32_t best = 0;
    for (int32_t i = 0; i < 8; i++) {
        float cd = vdot(desired, vnorm(v3(dirs[i][0], dirs[i][1], 0.f)));
        if (cd > maxd) { maxd = cd; best = i; }
    }
    a->act[0] = 1;
    a->act[1] = best;
    V3 fv = qrot(a->q, FWD);
    float ang = u_acos(clampf_(vdot(fv, vnorm(mv)), -1.f, 1.f));
    if (ang > K_PI / 8.f) {
        float cr = fv.x * mv.y - fv.y * mv.x;
        if (cr < 0.f) a->act[2] = -1;
        else if (cr > 0.f) a->act[2] = 1;
        else a->act[2] = 0;
    } else {
        a->act[2] = 0;
    }
}

/* fillObservationsSystem, game.cpp:1175-1461 */
typedef struct { float *o; int idx; } Obs;
static void put(Obs *s, float v) { s->o[s->idx++] = v; }
static void put3(Obs *s, V3 v) { put(s, v.x); put(s, v.y); put(s, v.z); }
static void put4(Obs *s, Q4 q) { put(s, q.w); put(s, q.x); put(s, q.y); put(s, q.z); }

static void put_other(Obs *s, const OAgent *o, V3 self_pos, V3 hoop, V3 ball_pos)
{
    V3 to = vsub(o->pos, self_pos);
    put3(s, o->pos);
    if (vlen2(to) > 1e-6f) put3(s, vnorm(to)); else put3(s, v3(0.f, 0.f, 0.f));
    put(s, vlen(to));
    put4(s, o->q);
    V3 f = qrot(o->q, FWD);
    put3(s, f);
    if (vlen2(o->vel) > 1e-6f) put3(s, vnorm(o->vel)); else put3(s, v3(0.f, 0.f, 0.f));
    put(s, vlen(o->vel));
    float d = 0.f;
    if (vlen2(o->vel) > 1e-6f) d = vdot(vnorm(o->vel), f);
    put(s, d);
    put(s, (d <= 0.8f) ? 0.1f : 1.f);
    V3 th = vsub(hoop, o->pos);
    float dh = vlen(th);
    if (dh > 1e-6f) put3(s, vnorm(th)); else put3(s, v3(0.f, 0.f, 0.f));
    put(s, dh);
    V3 tb = vsub(ball_pos, o->pos);
    float db = vlen(tb);
    if (db > 1e-6f) put3(s, vnorm(tb)); else put3(s, v3(0.f, 0.f, 0.f));
    put(s, db);
    put(s, (float)o->im_inb);
    put(s, o->cooldown);
    put(s, o->max_speed); put(s, o->quickness); put(s, o->shooting);
    put(s, o->ft); put(s, o->reaction); put(s, o->shot_pct);
    put(s, (float)o->points_worth);
    put(s, (float)o->has_ball);
}

static void sys_fill_obs(OWorld *w, int ai)
{
    OAgent *a = &w->ag[ai];
    const int n = G->n;
    Obs s; s.o = w->obs + (size_t)ai * G->obs_w; s.idx = 0;
    const OGame *g = &w->gs;
    const OBall *b = &w->ball;
    int32_t inbounder = -1;
    for (int i = 0; i < n; i++) if ((float)w->ag[i].im_inb > 0.5f) inbounder = w->ag[i].id;

    put(&s, g->clock); put(&s, g->shot); put(&s, g->period);
    put(&s, (float)g->inbounding); put(&s, g->inb_clock);
    if (a->team == 0) { put(&s, g->s0); put(&s, g->s1); }
    else { put(&s, g->s1); put(&s, g->s0); }
    put3(&s, b->pos); put3(&s, b->vel);
    put(&s, (float)b->grabbed); put(&s, (float)b->in_flight);
    put(&s, (float)b->shot_value); put(&s, (float)b->last_team);
    V3 att = (w->hoop[0].id != a->def_hoop) ? w->hoop[0].pos : w->hoop[1].pos;
    V3 dfn = (w->hoop[0].id == a->def_hoop) ? w->hoop[0].pos : w->hoop[1].pos;
    put3(&s, att); put3(&s, dfn);

    put3(&s, a->pos);
    put3(&s, v3(0.f, 0.f, 0.f));
    put(&s, 0.f);
    put4(&s, a->q);
    V3 f = qrot(a->q, FWD);
    put3(&s, f);
    if (vlen2(a->vel) > 1e-6f) put3(&s, vnorm(a->vel)); else put3(&s, v3(0.f, 0.f, 0.f));
    put(&s, vlen(a->vel));
    float d = 0.f;
    if (vlen2(a->vel) > 1e-6f) d = vdot(vnorm(a->vel), f);
    put(&s, d);
    put(&s, (d <= 0.8f) ? 0.1f : 1.f);
    V3 th = vsub(att, a->pos);
    float dh = vlen(th);
    if (dh > 1e-6f) put3(&s, vnorm(th)); else put3(&s, v3(0.f, 0.f, 0.f));
    put(&s, dh);
    V3 tb = vsub(b->pos, a->pos);
    float db = vlen(tb);
    if (db > 1e-6f) put3(&s, vnorm(tb)); else put3(&s, v3(0.f, 0.f, 0.f));
    put(&s, db);
    put(&s, (float)a->im_inb);
    put(&s, a->cooldown);
    put(&s, a->max_speed); put(&s, a->quickness); put(&s, a->shooting);
    put(&s, a->ft); put(&s, a->reaction); put(&s, a->shot_pct);
    put(&s, (float)a->points_worth);
    put(&s, (float)a->has_ball);

    int mates = 0, opps = 0;
    const int max_mates = n / 2 - 1, max_opps = n / 2;
    for (int i = 0; i < n; i++) {
        const OAgent *o = &w->ag[i];
        if (o->id == a->id) continue;
        if (o->team == a->team) {
            if (mates < max_mates) { put_other(&s, o, a->pos, att, b->pos); mates++; }
        } else {
            if (opps < max_opps) { put_other(&s, o, a->pos, dfn, b->pos); opps++; }
        }
    }
    if (mates < max_mates || opps < max_opps) EV(OR_EV_OBS_PADDED_ROW);
    for (int i = mates; i < max_mates; i++) for (int j = 0; j < 37; j++) put(&s, 0.f);
    for (int i = opps; i < max_opps; i++) for (int j = 0; j < 37; j++) put(&s, 0.f);
    for (int i = 0; i < n; i++) put(&s, (w->ag[i].id == b->holder) ? 1.f : 0.f);
    for (int i = 0; i < n; i++) put(&s, (w->ag[i].id == inbounder) ? 1.f : 0.f);
    for (; s.idx < G->obs_w; s.idx++) s.o[s.idx] = 0.f;
}

static void sys_reward(OWorld *w, OAgent *a) /* game.cpp:811-870 */
{
    int other = 0;
    for (int i = 0; i < G->n; i++) if (w->ag[i].id != a->id) other = i;
    float dist = vlen(vsub(w->ag[other].pos, a->pos));
    if ((float)a->team == w->gs.poss) {
        if (w->gs.clock > 5.f) {
            const OBall *b = &w->ball;
            if (b->shot_agent == a->id && b->going_in == 1) a->reward += (float)b->shot_value;
            else if (b->shot_agent == a->id && b->going_in == 0 && b->in_flight == 1) a->reward -= 1.f;
            a->reward += a->shot_pct;
        }
    } else {
        a->reward -= 1.f;
        a->reward = u_exp_add(a->reward, -0.4f * dist);
    }
}

static void step_world(OWorld *w) /* task graph order, game.cpp:1467-1523 */
{
    const int n = G->n;
    int i;
    for (i = 0; i < n; i++) sys_tick(w, &w->ag[i]);
    for (i = 0; i < n; i++) sys_action_mask(w, &w->ag[i]);
    for (i = 0; i < n; i++) sys_move_agent(w, &w->ag[i]);
    for (i = 0; i < n; i++) sys_grab(w, &w->ag[i]);
    for (i = 0; i < n; i++) sys_pass(w, &w->ag[i]);
    for (i = 0; i < n; i++) sys_shoot(w, &w->ag[i]);
    sys_move_ball(w);
    for (i = 0; i < n; i++) sys_shot_pct(w, &w->ag[i]);
    sys_score(w, &w->hoop[0]);
    sys_score(w, &w->hoop[1]);
    sys_out_of_bounds(w);
    sys_last_touch(w);
    sys_clock(w);
    sys_inbound_violation(w);
    sys_reset(w);
    for (i = 0; i < n; i++) sys_points_worth(w, &w->ag[i]);
    for (i = 0; i < n; i++) sys_collision(w, &w->ag[i]);
    for (i = 0; i < n; i++) sys_defense(w, &w->ag[i]);
    for (i = 0; i < n; i++) sys_fill_obs(w, i);
    for (i = 0; i < n; i++) sys_reward(w, &w->ag[i]);
}

/* ------------------------------------------------------------------ API */
int32_t oracle_obs_width(int32_t n)
{
    int32_t used = 61 + 38 * (n - 1) + 2 * n;
    int32_t w = (used + 3) & ~3;
    return w < 128 ? 128 : w;
}

void *oracle_create(const oracle_cfg *cfg)
{
    if (!cfg || cfg->num_agents < 2 || cfg->num_agents > MAXN || cfg->num_worlds < 1) return 0;
    init_court();
    Oracle *o = (Oracle *)calloc(1, sizeof(Oracle));
    o->cfg = *cfg;
    o->n = cfg->num_agents;
    o->obs_w = oracle_obs_width(o->n);
    o->width = (float)cfg->discrete_x / (float)1;  /* bindings.cpp:32-33, cellsPerMeter = 1 */
    o->height = (float)cfg->discrete_y / (float)1;
    o->flags = cfg->flags;
    o->w = (OWorld *)calloc((size_t)cfg->num_worlds, sizeof(OWorld));
    o->obs_store = (float *)calloc((size_t)cfg->num_worlds * o->n * o->obs_w, sizeof(float));
    G = o;
    g_math = cfg->math_mode;
    for (int64_t i = 0; i < cfg->num_worlds; i++) {
        o->w[i].obs = o->obs_store + (size_t)i * o->n * o->obs_w;
        generate_world(&o->w[i], cfg->world_offset + i);
    }
    return o;
}

void oracle_destroy(void *h)
{
    Oracle *o = (Oracle *)h;
    if (!o) return;
    if (G == o) G = 0;
    free(o->w); free(o->obs_store); free(o);
}

void oracle_step(void *h)
{
    Oracle *o = (Oracle *)h;
    G = o; g_math = o->cfg.math_mode;
    for (int64_t i = 0; i < o->cfg.num_worlds; i++) step_world(&o->w[i]);
}

static int64_t elems_per_world(const Oracle *o, int32_t id)
{
    const int n = o->n;
    switch (id) {
    case OR_EXPORT_RESET: return n;
    case OR_EXPORT_GAME_STATE: return 14;
    case OR_EXPORT_ACTION: return n * 6;
    case OR_EXPORT_ACTION_MASK: return n * 4;
    case OR_EXPORT_AGENT_POS: return n * 3;
    case OR_EXPORT_OBSERVATIONS: return (int64_t)n * o->obs_w;
    case OR_EXPORT_REWARD: return n;
    case OR_EXPORT_DONE: return n;
    case OR_EXPORT_AGENT_ENTITY_ID: return n;
    case OR_EXPORT_AGENT_POSSESSION: return n * 3;
    case OR_EXPORT_ORIENTATION: return n * 4;
    case OR_EXPORT_TEAM: return n * 5;
    case OR_EXPORT_AGENT_STATS: return n * 2;
    case OR_EXPORT_BALL_POS: return 3;
    case OR_EXPORT_BALL_PHYSICS: return 7;
    case OR_EXPORT_BALL_ENTITY_ID: return 1;
    case OR_EXPORT_BALL_GRABBED: return 2;
    case OR_EXPORT_BALL_VELOCITY: return 3;
    case OR_EXPORT_HOOP_POS: return 6;
    case OR_INTERNAL_AGENT_VELOCITY: return n * 3;
    case OR_INTERNAL_GRAB_COOLDOWN: return n;
    case OR_INTERNAL_CUR_STEP: return n;
    case OR_INTERNAL_INBOUNDING: return n * 2;
    case OR_INTERNAL_ATTRIBUTES: return n * 10;
    case OR_INTERNAL_WORLD_CLOCK: return 1;
    case OR_INTERNAL_RNG_COUNTER: return 1;
    default: return -1;
    }
}

int64_t oracle_export_bytes(void *h, int32_t id)
{
    Oracle *o = (Oracle *)h;
    int64_t e = elems_per_world(o, id);
    return e < 0 ? -1 : e * 4 * o->cfg.num_worlds;
}

typedef union { float f; int32_t i; uint32_t u; } W32;

static void xfer_world(Oracle *o, OWorld *w, int32_t id, W32 *p, int to_buf)
{
    const int n = o->n;
#define XF(dst, field) do { if (to_buf) (dst).f = (field); else (field) = (dst).f; } while (0)
#define XI(dst, field) do { if (to_buf) (dst).i = (field); else (field) = (dst).i; } while (0)
#define XU(dst, field) do { if (to_buf) (dst).u = (field); else (field) = (dst).u; } while (0)
    switch (id) {
    case OR_EXPORT_RESET: for (int i = 0; i < n; i++) XI(p[i], w->ag[i].reset); break;
    case OR_EXPORT_GAME_STATE: {
        OGame *g = &w->gs;
        XI(p[0], g->inbounding); XI(p[1], g->live); XF(p[2], g->period); XF(p[3], g->poss);
        XI(p[4], g->h0); XF(p[5], g->s0); XI(p[6], g->h1); XF(p[7], g->s1);
        XF(p[8], g->clock); XF(p[9], g->shot); XF(p[10], g->baskets); XF(p[11], g->oob);
        XF(p[12], g->inb_clock); XI(p[13], g->one_v_one);
    } break;
    case OR_EXPORT_ACTION: for (int i = 0; i < n; i++) for (int k = 0; k < 6; k++) XI(p[i * 6 + k], w->ag[i].act[k]); break;
    case OR_EXPORT_ACTION_MASK: for (int i = 0; i < n; i++) for (int k = 0; k < 4; k++) XI(p[i * 4 + k], w->ag[i].mask[k]); break;
    case OR_EXPORT_AGENT_POS: for (int i = 0; i < n; i++) { XF(p[i * 3], w->ag[i].pos.x); XF(p[i * 3 + 1], w->ag[i].pos.y); XF(p[i * 3 + 2], w->ag[i].pos.z); } break;
    case OR_EXPORT_OBSERVATIONS: for (int64_t k = 0; k < (int64_t)n * o->obs_w; k++) XF(p[k], w->obs[k]); break;
    case OR_EXPORT_REWARD: for (int i = 0; i < n; i++) XF(p[i], w->ag[i].reward); break;
    case OR_EXPORT_DONE: for (int i = 0; i < n; i++) XF(p[i], w->ag[i].done); break;
    case OR_EXPORT_AGENT_ENTITY_ID: for (int i = 0; i < n; i++) XI(p[i], w->ag[i].id); break;
    case OR_EXPORT_AGENT_POSSESSION: for (int i = 0; i < n; i++) { XI(p[i * 3], w->ag[i].has_ball); XI(p[i * 3 + 1], w->ag[i].ball_id); XI(p[i * 3 + 2], w->ag[i].points_worth); } break;
    case OR_EXPORT_ORIENTATION: for (int i = 0; i < n; i++) { XF(p[i * 4], w->ag[i].q.w); XF(p[i * 4 + 1], w->ag[i].q.x); XF(p[i * 4 + 2], w->ag[i].q.y); XF(p[i * 4 + 3], w->ag[i].q.z); } break;
    case OR_EXPORT_TEAM: for (int i = 0; i < n; i++) { XI(p[i * 5], w->ag[i].team); XF(p[i * 5 + 1], w->ag[i].color.x); XF(p[i * 5 + 2], w->ag[i].color.y); XF(p[i * 5 + 3], w->ag[i].color.z); XI(p[i * 5 + 4], w->ag[i].def_hoop); } break;
    case OR_EXPORT_AGENT_STATS: for (int i = 0; i < n; i++) { XF(p[i * 2], w->ag[i].st_points); XF(p[i * 2 + 1], w->ag[i].st_fouls); } break;
    case OR_EXPORT_BALL_POS: XF(p[0], w->ball.pos.x); XF(p[1], w->ball.pos.y); XF(p[2], w->ball.pos.z); break;
    case OR_EXPORT_BALL_PHYSICS: {
        OBall *b = &w->ball;
        XI(p[0], b->in_flight); XI(p[1], b->last_agent); XI(p[2], b->last_team); XI(p[3], b->shot_agent);
        XI(p[4], b->shot_team); XI(p[5], b->shot_value); XI(p[6], b->going_in);
    } break;
    case OR_EXPORT_BALL_ENTITY_ID: XI(p[0], w->ball.id); break;
    case OR_EXPORT_BALL_GRABBED: XI(p[0], w->ball.grabbed); XI(p[1], w->ball.holder); break;
    case OR_EXPORT_BALL_VELOCITY: XF(p[0], w->ball.vel.x); XF(p[1], w->ball.vel.y); XF(p[2], w->ball.vel.z); break;
    case OR_EXPORT_HOOP_POS: for (int h = 0; h < 2; h++) { XF(p[h * 3], w->hoop[h].pos.x); XF(p[h * 3 + 1], w->hoop[h].pos.y); XF(p[h * 3 + 2], w->hoop[h].pos.z); } break;
    case OR_INTERNAL_AGENT_VELOCITY: for (int i = 0; i < n; i++) { XF(p[i * 3], w->ag[i].vel.x); XF(p[i * 3 + 1], w->ag[i].vel.y); XF(p[i * 3 + 2], w->ag[i].vel.z); } break;
    case OR_INTERNAL_GRAB_COOLDOWN: for (int i = 0; i < n; i++) XF(p[i], w->ag[i].cooldown); break;
    case OR_INTERNAL_CUR_STEP: for (int i = 0; i < n; i++) XU(p[i], w->ag[i].cur_step); break;
    case OR_INTERNAL_INBOUNDING: for (int i = 0; i < n; i++) { XI(p[i * 2], w->ag[i].im_inb); XI(p[i * 2 + 1], w->ag[i].allowed_move); } break;
    case OR_INTERNAL_ATTRIBUTES: for (int i = 0; i < n; i++) {
        OAgent *a = &w->ag[i]; W32 *q = p + i * 10;
        XF(q[0], a->max_speed); XF(q[1], a->quickness); XF(q[2], a->shooting); XF(q[3], a->ft);
        XF(q[4], a->reaction); XF(q[5], a->target.x); XF(q[6], a->target.y); XF(q[7], a->target.z);
        XF(q[8], a->shot_pct);
        if (to_buf) q[9].f = 0.f; /* pad */
    } break;
    case OR_INTERNAL_WORLD_CLOCK: XI(p[0], w->reset_now); break;
    case OR_INTERNAL_RNG_COUNTER: XU(p[0], w->ctr); break;
    default: break;
    }
#undef XF
#undef XI
#undef XU
}

void oracle_export(void *h, int32_t id, void *out)
{
    Oracle *o = (Oracle *)h;
    int64_t e = elems_per_world(o, id);
    if (e < 0) return;
    W32 *p = (W32 *)out;
    for (int64_t i = 0; i < o->cfg.num_worlds; i++) xfer_world(o, &o->w[i], id, p + i * e, 1);
}

void oracle_import(void *h, int32_t id, const void *in)
{
    Oracle *o = (Oracle *)h;
    int64_t e = elems_per_world(o, id);
    if (e < 0) return;
    W32 *p = (W32 *)in;
    for (int64_t i = 0; i < o->cfg.num_worlds; i++) xfer_world(o, &o->w[i], id, p + i * e, 0);
}

void oracle_random_actions(void *h, uint32_t seed, uint32_t step)
{
    Oracle *o = (Oracle *)h;
    for (int64_t i = 0; i < o->cfg.num_worlds; i++) {
        uint32_t gw = (uint32_t)(o->cfg.world_offset + i);
        for (int a = 0; a < o->n; a++) {
            uint32_t r[2];
            oracle_threefry2x32(seed, step, gw, (uint32_t)a, r);
            int32_t *act = o->w[i].ag[a].act;
            act[0] = (int32_t)(r[0] & 1u);
            act[1] = (int32_t)((r[0] >> 1) & 7u);
            act[2] = (int32_t)(((r[0] >> 4) & 0xFFFFu) % 3u);
            act[3] = (int32_t)((r[0] >> 20) & 1u);
            act[4] = (int32_t)((r[0] >> 21) & 1u);
            act[5] = (int32_t)((r[0] >> 22) & 1u);
        }
    }
}

double oracle_run_random(void *h, int32_t steps, uint32_t seed, uint32_t step0)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int32_t s = 0; s < steps; s++) {
        oracle_random_actions(h, seed, step0 + (uint32_t)s);
        oracle_step(h);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

int32_t oracle_shot_point_value(float px, float py, float pz, float hx, float hy, float hz)
{
    init_court();
    return shot_value(v3(px, py, pz), v3(hx, hy, hz));
}

void oracle_events(void *h, int64_t out[OR_NUM_EVENTS])
{
    Oracle *o = (Oracle *)h;
    for (int k = 0; k < OR_NUM_EVENTS; k++) out[k] = o->ev[k];
}

void oracle_rotate_vec(const float q[4], const float v[3], float out[3])
{
    Q4 qq; qq.w = q[0]; qq.x = q[1]; qq.y = q[2]; qq.z = q[3];
    V3 r = qrot(qq, v3(v[0], v[1], v[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

void oracle_court_constants(float out[8])
{
    init_court();
    out[0] = g_world_w; out[1] = g_world_h; out[2] = g_cminx; out[3] = g_cmaxx;
    out[4] = g_cminy; out[5] = g_cmaxy; out[6] = K_TS; out[7] = K_PI;
}
