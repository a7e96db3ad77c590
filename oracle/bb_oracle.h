/*
 * bb_oracle.h -- CPU oracle for the batched basketball step.
 *
 * TEST INFRASTRUCTURE ONLY.  This is a plain-C restatement of the reference's
 * per-step task graph (davidj24/madrona_basketball, src/game.cpp:1463-1526,
 * src/gen.cpp, src/helper.cpp).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker / the timed
 * CPU baseline.  The product (madrona_basketball_amd) never links it.
 *
 * Parity status: PARTIALLY PINNED.  The reference cannot be built here (its
 * Madrona submodule is not vendored), so this restatement is pinned by the
 * known answers the reference's own files hold (src/constants.py values,
 * scripts/ppo.py:117 hoop positions, scripts/viewer.py:59-65 rotate_vec,
 * the clock horizon implied by src/constants.hpp:11-13) -- see
 * tests/golden/.  Madrona-internal arithmetic (RNG bit stream,
 * Vector3::normalize, entity-id assignment) is unpinned and fixed by the
 * build's own definitions, documented in DESIGN.md.
 */
#ifndef BB_ORACLE_H
#define BB_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Export ids: src/types.hpp:10-42 order, plus build-internal state ids. */
enum {
    OR_EXPORT_RESET = 0, OR_EXPORT_GAME_STATE, OR_EXPORT_ACTION, OR_EXPORT_ACTION_MASK,
    OR_EXPORT_AGENT_POS, OR_EXPORT_OBSERVATIONS, OR_EXPORT_REWARD, OR_EXPORT_DONE,
    OR_EXPORT_AGENT_ENTITY_ID, OR_EXPORT_AGENT_POSSESSION, OR_EXPORT_ORIENTATION,
    OR_EXPORT_TEAM, OR_EXPORT_AGENT_STATS, OR_EXPORT_BALL_POS, OR_EXPORT_BALL_PHYSICS,
    OR_EXPORT_BALL_ENTITY_ID, OR_EXPORT_BALL_GRABBED, OR_EXPORT_BALL_VELOCITY,
    OR_EXPORT_HOOP_POS,
    OR_INTERNAL_AGENT_VELOCITY = 32, OR_INTERNAL_GRAB_COOLDOWN, OR_INTERNAL_CUR_STEP,
    OR_INTERNAL_INBOUNDING, OR_INTERNAL_ATTRIBUTES, OR_INTERNAL_WORLD_CLOCK,
    OR_INTERNAL_RNG_COUNTER
};

/* flags */
#define OR_FLAG_PER_WORLD_RNG 0x1u  /* key each world's RNG by its global index */
#define OR_FLAG_NO_TAG_MASK   0x2u  /* skip the tag override (game.cpp:526-528) */
#define OR_FLAG_FULL_GAME     0x4u  /* isOneOnOne = 0 (constants.hpp:27 set to 0) */

/* math modes */
#define OR_MATH_CR   0  /* float transcendental f(x) := (float) libm_double(x)  */
#define OR_MATH_LIBM 1  /* literal glibc float calls, exactly as the reference */
#define OR_MATH_LIBM_FLOAT 2  /* as LIBM, but game.cpp:746,808,868's unqualified acos / erf / exp bound
                                 to the float overloads (acosf / erff / expf): the unpinned other reading */

typedef struct oracle_cfg {
    int32_t num_agents;
    int64_t num_worlds;
    int32_t discrete_x, discrete_y;
    float start_x, start_y;
    uint32_t seed;
    uint32_t flags;
    int64_t world_offset;
    int32_t math_mode;
} oracle_cfg;

void *oracle_create(const oracle_cfg *cfg);
void oracle_destroy(void *h);
void oracle_step(void *h);
int32_t oracle_obs_width(int32_t num_agents);
/* Copy one export / internal column in the reference tensor layout. */
int64_t oracle_export_bytes(void *h, int32_t id);
void oracle_export(void *h, int32_t id, void *out);
/* Overwrite one column from the reference tensor layout (writable tensors). */
void oracle_import(void *h, int32_t id, const void *in);
/* Synthetic random actions (bench/test workload): threefry2x32-20 of
 * key {seed, step}, counter {global world, agent}. */
void oracle_random_actions(void *h, uint32_t seed, uint32_t step);
/* Timed loop used by bench.py's cpu_baseline leg; returns wall seconds. */
double oracle_run_random(void *h, int32_t steps, uint32_t seed, uint32_t step0);
/* Cumulative event counts since creation: which rare branches a run went
 * through (coverage assertions of the parity tests). */
enum {
    OR_EV_SHOT = 0,            /* holder released a shot (shootSystem, game.cpp:273-407) */
    OR_EV_SHOT_GOING_IN,       /* ... on a going-in line */
    OR_EV_MAKE,                /* scoreSystem hit (game.cpp:873-953) */
    OR_EV_OOB_1V1,             /* 1v1 out of bounds: -100 + reset (game.cpp:1055-1113) */
    OR_EV_OOB_TURNOVER,        /* full-game out-of-bounds turnover (game.cpp:1083-1111) */
    OR_EV_TAG,                 /* contact against the possessing team (game.cpp:537-648) */
    OR_EV_CONTACT,             /* any SAT contact */
    OR_EV_INBOUND_START,       /* assignInbounder assigned an agent (game.cpp:14-53) */
    OR_EV_INBOUND_VIOLATION,   /* 5-s inbound violation (game.cpp:1116-1157) */
    OR_EV_PERIOD_ADVANCE,      /* end-of-period branch of resetWorld (gen.cpp:221-236) */
    OR_EV_GAME_END,            /* game-over branch of resetWorld (gen.cpp:221-236) */
    OR_EV_WORLD_RESET,         /* resetSystem ran resetWorld (game.cpp:957-967) */
    OR_EV_CLOCK_EXPIRY,        /* clockSystem +10 and reset (game.cpp:992-1030) */
    OR_EV_GRAB,                /* grab / steal picked up the ball (game.cpp:164-239) */
    OR_EV_PASS,                /* pass released the ball (game.cpp:243-270) */
    OR_EV_DEFENDER_GRAB_RESET, /* 1v1 defender grab -> reset (game.cpp:164-239) */
    OR_EV_OBS_PADDED_ROW,      /* observation row with empty mate/opponent slots (game.cpp:1428-1437) */
    OR_NUM_EVENTS
};
void oracle_events(void *h, int64_t out[OR_NUM_EVENTS]);

/* Exposed primitives for known-answer tests. */
void oracle_threefry2x32(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t out[2]);
int32_t oracle_shot_point_value(float px, float py, float pz, float hx, float hy, float hz);
void oracle_rotate_vec(const float q[4], const float v[3], float out[3]);
void oracle_court_constants(float out[8]);

#ifdef __cplusplus
}
#endif
#endif
