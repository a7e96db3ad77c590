// bb_kernels.hip -- gfx950 step kernel of the basketball simulator; compiled
// once per agent count (-DBB_N=2,4,6,8,10).
//
// k_step<N>: one wave = one 64-lane workgroup; at N = 2 and 4 one lane per
// agent (64/N worlds per wave), otherwise one lane per world.
//   1. every lane loads its world's columns (16/8-byte vector loads where the
//      per-world chunk allows) into a register-resident World<N>;
//   2. systems 1-17 of src/game.cpp:1463-1526 run on registers (bb_sim.h);
//      with agent lanes the per-agent systems are split over the world's
//      lanes and their results exchanged by DPP;
//   3. rewardSystem, then the state columns are stored;
//   4. fillObservations (game.cpp:1175-1461): rows go into an LDS tile
//      (conflict-free ds_write_b128, row stride 4 mod 8 dwords); the wave
//      then stores the 64 rows -- consecutive in memory -- as consecutive
//      16-byte pieces (whole 128-byte lines per instruction instead of 64
//      scattered ones).
// Replaces the reference's 19 ParallelFor megakernel nodes + 3 sort nodes per
// step (src/game.cpp:1467-1523, src/sim.cpp:99-124) with one launch.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdlib>
#include <type_traits>
#include "bb_launch.h"
#include "bb_policy_dev.h"
#include "bb_sim.h"

#ifndef BB_N
#error "compile bb_kernels.hip with -DBB_N=<agents>"
#endif

namespace bb {

constexpr int WAVE = 64;

// Cache policy of the observation-row stores (the bulk of a step's bytes):
// -1 a plain global store; otherwise a buffer store with these aux bits
// (gfx950: 1 sc0, 2 nt, 16 sc1 -- sc1 writes the line through and drops it
// from the XCD's L2, so no dirty row lines are left for the end-of-kernel
// write-back).
#ifndef BB_STEP_AUX
// k_step, rows cache-resident: write-through (sc1), which leaves the kernel
// fewer dirty L2 lines to settle at its end -- measured 8 192 worlds 11.65 ->
// 11.13 us, 16 384 12.93 -> 12.15, 32 768 15.7 -> 15.4 (profiles/r03/
// k_store_policy_small_ab.txt), 65 536 equal (r02 o_store_policy_ab.txt);
// nt is slower at every cache-resident size.
#define BB_STEP_AUX 16
#endif
#ifndef BB_COL_AUX
#define BB_COL_AUX -1  // k_step<2>, state column stores (vector chunks)
#endif
#ifndef BB_LINES_AUX
#define BB_LINES_AUX 2  // k_step, state beyond the Infinity Cache
#endif
#ifndef BB_ROLLOUT_AUX
#define BB_ROLLOUT_AUX 2  // k_rollout: rows into a fresh K-step buffer
#endif
#ifndef BB_SHARED_AUX
#define BB_SHARED_AUX -1  // N >= 4, rows and columns while the step fits the cache
#endif
// Wave priority (s_setprio) while a wave of the shared-world kernel emits its
// rows / issues its state loads: memory work of one wave ahead of the
// systems of the others on its SIMD.
#ifndef BB_PRIO_ROWS
#define BB_PRIO_ROWS 0
#endif
#ifndef BB_PRIO_LOAD
#define BB_PRIO_LOAD 0
#endif
#ifndef BB_SHARED_BEYOND_AUX
#define BB_SHARED_BEYOND_AUX 2  // N >= 4 beyond the cache: rows
#endif
#ifndef BB_SHARED_BEYOND_COL_AUX
#define BB_SHARED_BEYOND_COL_AUX 2  // N >= 4 beyond the cache: state columns
#endif

// The erf Taylor table (bb_math.h) copied to LDS by the workgroup's one
// wave (k_rollout): shotPercentage's per-lane coefficient reads become LDS
// reads instead of memory loads, which, issued after a step's stores, would
// wait for all of them (the vector-memory counter retires in order).  k_step
// reads the table from memory: there no store precedes the read, and the
// copy's wait would serialise the state loads.
constexpr int ERF_WORDS = bbm::ERF_TK * (bbm::ERF_TD + 1);
#ifndef BB_ERF_LDS
#define BB_ERF_LDS 1
#endif
__device__ __forceinline__ const double *erf_table_lds()
{
    if constexpr (!BB_ERF_LDS) return &bbm::ERF_TAYLOR[0][0];
    __shared__ double tab[ERF_WORDS];
    const double *g = &bbm::ERF_TAYLOR[0][0];
#pragma unroll
    for (int j = 0; j < (ERF_WORDS + WAVE - 1) / WAVE; j++) {
        const int i = j * WAVE + (int)(threadIdx.x % WAVE);  // (every wave writes the whole table)
        if (i < ERF_WORDS) tab[i] = g[i];
    }
    return tab;
}

// Ordering of LDS words written and read by different lanes of one wave (a
// wave's LDS operations execute in order): keeps the compiler from moving
// them across each other.
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier ordering LDS only: a release fence at workgroup scope
// over global memory too (__syncthreads) would wait for the wave's
// outstanding global stores before every hand-off.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int N>
struct ObsTile {
    static constexpr int QW = (obs_used(N) + 3) / 4;  // float4 pieces of a used row
    static constexpr int RS = QW * 4 + 4;             // LDS row stride (floats): == 4 mod 8
    // LDS-staged rows only while the tile leaves room for >= 2 waves per CU
    static constexpr bool STAGED = (WAVE * RS * 4) <= 64 * 1024;
    static constexpr int FLOATS = STAGED ? WAVE * RS : 4;
};

// Lanes per world.  With one lane per agent (N = 2, 4) each lane holds the
// whole world and runs the world-level systems, but computes only its own
// agent's share of the per-agent systems (move, shot percentage, points
// worth, defence), reward, intrinsic observation block and observation row;
// the other agents' results come from the neighbouring lanes by DPP.
#ifndef BB_AGENT_LANES
#define BB_AGENT_LANES 1
#endif
template <int N>
struct Lanes {
    // SHARED: one lane per agent, the world's state in LDS shared by its N
    // lanes (pick_by indexes directly from the same N on, bb_sim.h)
    static constexpr bool SHARED = N >= LDS_WORLD_MIN_N;
    static constexpr int LPW = SHARED ? N : ((BB_AGENT_LANES && (N == 2 || N == 4)) ? N : 1);
    static constexpr int WPB = WAVE / LPW;  // worlds per 64-lane workgroup
};

// Row tile of the agent-lane kernel: the row is emitted in PH passes of QP
// float4 pieces so the tile stays ~16 KB (>= 8 waves per CU).
#ifndef BB_OBS_WRITE_ALIGN
#define BB_OBS_WRITE_ALIGN 16  // bytes: row writes end on this boundary (zero pieces added)
#endif
#ifndef BB_OBS_PHASE_PIECES
#define BB_OBS_PHASE_PIECES 15  // at most this many 16-byte pieces of a row per pass
#endif
// ALIGN: row writes end on this byte boundary (zero pieces added);
// MAXP: at most this many 16-byte pieces of a row per pass; ROUND: a pass
// holds a multiple of this many pieces (4: passes split rows on 64-byte
// segment boundaries; diagnostic variants).
#ifndef BB_OBS_PHASE_ROUND
#define BB_OBS_PHASE_ROUND 1
#endif
template <int N, int ALIGN = BB_OBS_WRITE_ALIGN, int MAXP = BB_OBS_PHASE_PIECES, int STORE_AUX = BB_STEP_AUX,
          int ROUND = BB_OBS_PHASE_ROUND>
struct PhasedTile {
    static constexpr int AUX = STORE_AUX;  // cache policy of the row stores (row_store)
    static constexpr int QU = (obs_used(N) + 3) / 4;  // pieces holding row values
    static constexpr int QA = (QU * 16 + ALIGN - 1) / ALIGN * ALIGN / 16;
    static constexpr int QW = QA < obs_width(N) / 4 ? QA : obs_width(N) / 4;  // pieces written
    static constexpr int PH = (QW + MAXP - 1) / MAXP;
    static constexpr int QP = ((QW + PH - 1) / PH + ROUND - 1) / ROUND * ROUND;
    static constexpr int RS = QP * 4 + (QP % 2 == 0 ? 4 : 0);  // == 4 mod 8 dwords
    static constexpr int FLOATS = WAVE * RS;
};

// k_rollout's rows go to a fresh [K][W][N][OBSW] buffer far larger than the
// Infinity Cache: every 128-byte line is written whole by one pass (passes of
// 16 pieces = 2 lines per row, the zero tail included), since lines left
// partial by a pass reach memory as partial writes (measured: 25.7 -> 18.1 us
// per step at 65 536 worlds).  k_step's 64 MiB rows stay cache-resident,
// where the 416 written bytes of 2 x 13 pieces are cheaper.
#ifndef BB_LINES_ALIGN
#define BB_LINES_ALIGN 128  // beyond-cache row writes end on this byte boundary
#endif
#ifndef BB_LINES_MAXP
#define BB_LINES_MAXP 16
#endif
template <int N>
using RolloutTile = PhasedTile<N, BB_LINES_ALIGN, BB_LINES_MAXP, BB_ROLLOUT_AUX, 1>;

// k_step's tile.  LINES (state beyond the Infinity Cache): whole 128-byte
// lines per pass, zero tail included, like k_rollout -- at 262 144 worlds
// 99.3 -> 88.0 us per step (partial lines reach HBM as partial writes);
// otherwise 2 x 13 pieces (416 written bytes per row), cheaper while the rows
// stay cache-resident (65 536 worlds: 21.95 vs 22.14 us).
template <int N, bool LINES>
using StepTile = typename std::conditional<LINES, PhasedTile<N, BB_LINES_ALIGN, BB_LINES_MAXP, BB_LINES_AUX, 1>, PhasedTile<N>>::type;

// RowSink restricted to floats [LO, HI) of the row; `row` points at float LO.
// Indices are compile-time after unrolling, so the window test folds away and
// values outside the window are never computed.
template <int LO, int HI>
struct WindowSink {
    float *row;
    float b0, b1, b2, b3;
    int idx;
    __device__ void put(float v)
    {
        if (idx >= LO && idx < HI) {
            switch (idx & 3) {
            case 0: b0 = v; break;
            case 1: b1 = v; break;
            case 2: b2 = v; break;
            default: b3 = v; store_f4(row + ((idx & ~3) - LO), b0, b1, b2, b3); break;
            }
        }
        idx++;
    }
    __device__ void put3(F3 v) { put(v.x); put(v.y); put(v.z); }
    __device__ void put4(Q4 q) { put(q.w); put(q.x); put(q.y); put(q.z); }
    __device__ void finish() { while (idx & 3) put(0.f); }
};

// DPP quad_perm controls: lane k of each G-lane group (G = 2, 4) reads
// lane J of its group (bcast), or the lane of the agent in slot T of lane
// k's agent view (view).
template <int G, int J>
constexpr int bcast_ctrl()
{
    int c = 0;
    for (int l = 0; l < 4; l++) c |= ((l / G) * G + J) << (2 * l);
    return c;
}
template <int G, int T>
constexpr int view_ctrl()
{
    int c = 0;
    for (int l = 0; l < 4; l++) c |= ((l / G) * G + view_source<G>(T, l % G)) << (2 * l);
    return c;
}

template <int CTRL, class T>
__device__ __forceinline__ T lane_dpp(const T &x)
{
    static_assert(sizeof(T) % 4 == 0, "32-bit words");
    constexpr int NW = sizeof(T) / 4;
    int in[NW], out[NW];
    __builtin_memcpy(in, &x, sizeof(T));
#pragma unroll
    for (int q = 0; q < NW; q++) out[q] = __builtin_amdgcn_update_dpp(0, in[q], CTRL, 0xF, 0xF, false);
    T r;
    __builtin_memcpy(&r, out, sizeof(T));
    return r;
}

// Value of `x` in lane (lane & ~(G-1)) + J.
template <int G, int J, class T>
__device__ __forceinline__ T lane_bcast(const T &x)
{
    static_assert(G == 2 || G == 4, "quad groups");
    return lane_dpp<bcast_ctrl<G, J>()>(x);
}

// out[j] = agent j's value (creation order), from the world's G lanes.
template <int G, class T, int J = 0>
__device__ __forceinline__ void lane_gather(const T &mine, T (&out)[G])
{
    out[J] = lane_bcast<G, J>(mine);
    if constexpr (J + 1 < G) lane_gather<G, T, J + 1>(mine, out);
}

// out[t] = value of the agent in slot t of this lane's agent view
// (view_source): slot 0 is the lane itself, one DPP per further slot.
template <int G, class T, int J = 1>
__device__ __forceinline__ void lane_gather_view(const T &mine, T (&out)[G])
{
    if constexpr (J == 1) out[0] = mine;
    if constexpr (J < G) {
        out[J] = lane_dpp<view_ctrl<G, J>()>(mine);
        lane_gather_view<G, T, J + 1>(mine, out);
    }
}

// MODE_TRACE: lane 0 of each wave records the constant-rate clock at the
// phase boundaries -- 0 start, 1 state loaded, 2-7 after groups of systems
// (bb_sim.h step_world_pre_obs marks), 8 state stored, 9 end -- and in slot
// 10 how many of the wave's lanes belong to a world reset this step.
constexpr int TRACE_POINTS = 12;
template <int MODE>
__device__ __forceinline__ void trace_point(const Params &p, int point)
{
    if constexpr (MODE == MODE_TRACE) {
        if (point == 1) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t t = wall_clock64();
        if (threadIdx.x == 0) p.diag_ts[(int64_t)blockIdx.x * TRACE_POINTS + point] = t;
    }
}
template <int MODE, int N>
__device__ __forceinline__ void trace_resets(const Params &p, bool active, const World<N> &s)
{
    if constexpr (MODE == MODE_TRACE) {
        const uint64_t m = __ballot(active && s.done[0] != 0.f);  // resetWorld sets Done = 1
        if (threadIdx.x == 0) p.diag_ts[(int64_t)blockIdx.x * TRACE_POINTS + 10] = (uint64_t)__popcll(m);
    }
}

// Agent policy of the agent-lane kernel (see EachAgent in bb_sim.h).  Called
// at the top level of step_world_pre_obs, where the N lanes of a world are
// converged.
// OWN_APPLY: the world lives in LDS shared by its G lanes (the N = 4
// shared-world kernel), so in each() a lane applies only its own agent's
// result; with the world in every lane's registers each lane applies all G.
template <int G, int MODE, bool OWN_APPLY = false>
struct LaneAgents {
    int k;
    const Params *p;
    template <class T, int N, class F>
    __device__ void all(F f, T (&out)[N]) const
    {
        static_assert(N == G, "one lane per agent");
        lane_gather<G>(f(k), out);
    }
    template <int N, class F, class P>
    __device__ void each(F f, P apply) const
    {
        static_assert(N == G, "one lane per agent");
        if constexpr (OWN_APPLY) {
            apply(k, f(k));
            // the next system reads the other lanes' LDS writes: a workgroup
            // barrier orders them (the block is one wave, so it costs ~nothing)
            __syncthreads();
        } else {
            decltype(f(0)) out[G];
            lane_gather<G>(f(k), out);
#pragma unroll
            for (int i = 0; i < G; i++) apply(i, out[i]);
        }
    }
    __device__ void mark(int point) const { trace_point<MODE>(*p, point); }
};

// Copy the wave's 64 staged rows (tile row r -> obs row row0 + r*RSTR) as
// consecutive 16-byte pieces: tile piece q -> row piece Q0 + q, q < QN.
// Rows whose bit is clear in `staged` were written directly or belong to no
// world.  Pieces f = it*64 + lane: every LDS read of a batch is issued before
// its stores, addresses are 32-bit offsets from the wave's first row.
typedef float vf4 __attribute__((ext_vector_type(4)));  // plain 16-byte loads/stores
typedef uint32_t vu4 __attribute__((ext_vector_type(4)));

template <int AUX>
__device__ __forceinline__ void row_store(char *base, uint32_t off, vf4 v)
{
    if constexpr (AUX < 0) {
        *(vf4 *)(base + off) = v;
    } else {
        // base is wave-uniform (the wave's first row): one descriptor per wave
        const uint64_t b = (uint64_t)base;
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
        char *ub = (char *)(((uint64_t)hi << 32) | lo);
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(ub, 0, 0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(vu4, v), rs, (int)off, 0, AUX);
    }
}

// The record of agent `agent`'s rows (Params::rec_obs, N = 2): row r of the
// wave's tile (world r / N, agent r % N) also goes to base + (r / N) * 512
// (+ the pass's piece offset); base == nullptr: no record.  mirror: every
// row also to base at its own offset (a K-step rollout's last step: the rows
// into the sim's observation tensor as well as the recorded buffer).
struct RecRows {
    char *base;
    int agent;
    bool only;  // the agent's rows into the record only (Params::rec_only)
    bool mirror = false;
};
#ifndef BB_REC_AUX
#define BB_REC_AUX 2  // record rows: non-temporal (a fresh [K][W][128] buffer, beyond the cache for K >= 8)
#endif

template <int N, int QT, int RS, int Q0, int QN, int RSTR, bool ALL, int QZ, int AUX>
__device__ __forceinline__ void flush_rows(const float *tile, char *base, uint64_t staged, int lane, RecRows rec)
{
    // pieces q >= QZ of this pass are zeros (row padding), not read from the tile
    constexpr int OW = obs_width(N);
    constexpr int DR = WAVE / QT, DQ = WAVE % QT;  // advance of f by 64
    constexpr int BS = QT <= 16 ? QT : (QT + 1) / 2;
    int r = lane / QT, q = lane - (lane / QT) * QT;
#pragma unroll
    for (int b0 = 0; b0 < QT; b0 += BS) {
        vf4 v[BS];
        uint32_t go[BS], ro[BS];
        bool ok[BS], rk[BS], sk[BS];
#pragma unroll
        for (int j = 0; j < BS; j++) {
            if (b0 + j < QT) {
                ok[j] = (QN == QT || q < QN) && (ALL || ((staged >> r) & 1ull));
                go[j] = (uint32_t)(r * (RSTR * OW * 4) + q * 16);
                rk[j] = ok[j] && (rec.mirror || (r % N) == rec.agent);
                sk[j] = ok[j] && !(rec.only && (r % N) == rec.agent);
                ro[j] = rec.mirror ? go[j] : (uint32_t)((r / N) * (OW * 4) + q * 16);
                if (ok[j]) {
                    v[j] = *(const vf4 *)(tile + r * RS + 4 * q);
                    if (QZ < QN && q >= QZ) v[j] = vf4{0.f, 0.f, 0.f, 0.f};
                }
                r += DR;
                q += DQ;
                if (q >= QT) { q -= QT; r += 1; }
            }
        }
#pragma unroll
        for (int j = 0; j < BS; j++)
            if (b0 + j < QT && sk[j]) row_store<AUX>(base, go[j], v[j]);
        if (rec.base) {  // wave-uniform
#pragma unroll
            for (int j = 0; j < BS; j++)
                if (b0 + j < QT && rk[j]) row_store<BB_REC_AUX>(rec.base, ro[j], v[j]);
        }
    }
}

template <int N, int QT, int RS, int Q0, int QN, int RSTR, int QZ = QN, int AUX = -1>
__device__ __forceinline__ void flush_tile(const float *tile, float *obs, int64_t row0, uint64_t staged, int lane,
                                           RecRows rec = RecRows{nullptr, 0, false})
{
    char *base = (char *)(obs + row0 * obs_width(N) + 4 * Q0);  // wave-uniform
    if (rec.base) rec.base += 16 * Q0;
    if (staged == ~0ull) flush_rows<N, QT, RS, Q0, QN, RSTR, true, QZ, AUX>(tile, base, staged, lane, rec);
    else flush_rows<N, QT, RS, Q0, QN, RSTR, false, QZ, AUX>(tile, base, staged, lane, rec);
}

struct Intrinsic {
    float v[INTRINSIC];
};

// Pass PHASE of the lane's row into its tile row (shared path or fast path).
template <int N, class T, int PHASE>
__device__ __forceinline__ void emit_phase(const World<N> &v, const Ctx &c, const SharedObs<N> &sh, bool share,
                                           float *trow, int32_t ib)
{
    constexpr int LO = PHASE * T::QP * 4, HI = LO + T::QP * 4;
    WindowSink<LO, HI> o;
    o.row = trow; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
    if (share) emit_row_shared(v, c, sh, 0, o, ib);
    else emit_row_fast(v, c, 0, o, ib);
}

template <int N, int MODE, class T, int PHASE = 0>
__device__ __forceinline__ void obs_phases(const World<N> &v, const Ctx &c, const SharedObs<N> &sh, bool share,
                                           bool fast, float *tile, float *obs, int64_t row0, int lane, int32_t ib,
                                           RecRows rec = RecRows{nullptr, 0, false})
{
    if (fast) emit_phase<N, T, PHASE>(v, c, sh, share, tile + lane * T::RS, ib);
    __syncthreads();
    constexpr int Q0 = PHASE * T::QP, QN = (T::QW - Q0 < T::QP) ? T::QW - Q0 : T::QP;
    constexpr int QZ = T::QU - Q0 < 0 ? 0 : (T::QU - Q0 < QN ? T::QU - Q0 : QN);
    flush_tile<N, T::QP, T::RS, Q0, QN, 1, QZ, T::AUX>(tile, obs, row0, __ballot(fast), lane, rec);
    if constexpr (PHASE + 1 < T::PH) {
        __syncthreads();
        obs_phases<N, MODE, T, PHASE + 1>(v, c, sh, share, fast, tile, obs, row0, lane, ib, rec);
    }
}

struct LaneOrig {
    WorldOrig world;
    OrigAgent agent;
};
static_assert(sizeof(LaneOrig) <= 4 * 52, "fits a row of the observation tile");

// Words a lane parks in the observation tile until its observation pass,
// word-major (word i of lane l at tile[i * WAVE + l]): each ds_write_b32 /
// ds_read_b32 then covers 32 consecutive banks per lane group.  Lane-major at
// the tile's row stride (52 or 68 dwords, 4 mod 8) they were 4-way bank
// conflicts, most of k_step<2>'s SQ_LDS_BANK_CONFLICT.
template <class X>
__device__ __forceinline__ void park_words(float *tile, int lane, const X &x)
{
    static_assert(sizeof(X) % 4 == 0, "whole words");
    uint32_t u[sizeof(X) / 4];
    __builtin_memcpy(u, &x, sizeof(X));
    uint32_t *t = (uint32_t *)tile;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(X) / 4); i++) t[i * WAVE + lane] = u[i];
}
template <class X>
__device__ __forceinline__ X unpark_words(const float *tile, int lane)
{
    uint32_t u[sizeof(X) / 4];
    const uint32_t *t = (const uint32_t *)tile;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(X) / 4); i++) u[i] = t[i * WAVE + lane];
    X x;
    __builtin_memcpy(&x, u, sizeof(X));
    return x;
}

// Observation rows of the agent-lane kernel into obs (a [W][N][OBSW] base):
// the lane's intrinsic block, exchanged with the world's lanes by DPP, then
// the row through the LDS tile (fast rows) or directly (slow rows).
// ib / share: inbounder_id and obs_sharable of the world in creation order.
// The row sources of the lane's agent (slot 0 of its view v): the intrinsic
// blocks of every agent of the world (its own computed here, the others' by
// DPP from their lanes) and the directions / distances to the others.
template <int N>
__device__ __forceinline__ void lane_shared_obs(const World<N> &v, const Ctx &c, bool active, SharedObs<N> &sh)
{
    if (active) {
        Intrinsic mine, slot[N];
        {
            ArraySink<INTRINSIC> o;
            o.idx = 0;
            emit_intrinsic(v, o, 0, attacking_hoop(v, c, 0));
#pragma unroll
            for (int q = 0; q < INTRINSIC; q++) mine.v[q] = o.v[q];
        }
        lane_gather_view<N>(mine, slot);
#pragma unroll
        for (int t = 0; t < N; t++)
#pragma unroll
            for (int q = 0; q < INTRINSIC; q++) sh.intr[t].v[q] = slot[t].v[q];
#pragma unroll
        for (int t = 1; t < N; t++) {
            const F3 to = v.pos(t) - v.pos(0);
            const float l2 = len2(to);
            const float r = 1.0f / bbm::sqrtf_(l2);  // the factor norm() applies
            sh.rdir[0][t] = l2 > 1e-6f ? to * r : f3(0.f, 0.f, 0.f);
            sh.rlen[0][t] = bbm::sqrtf_(l2);
        }
    }
}

// mirror_sim (wave-uniform; not with REC): every row also into the sim's own
// observation tensor (c.p->c.obs), obs being a recorded buffer.
template <int N, int MODE, class T = PhasedTile<N>, bool REC = false>
__device__ __forceinline__ void agent_lane_obs(const World<N> &v, const Ctx &c, int32_t ib, bool share, int k,
                                               int lane, int64_t w0, int64_t w, bool active, float *tile, float *obs,
                                               bool mirror_sim = false)
{
    constexpr int OW = obs_width(N);
    SharedObs<N> sh;
    lane_shared_obs(v, c, active, sh);
    float *grow = obs + (w * N + k) * (int64_t)OW;
    const bool fast = active && canonical_slots(v, 0);
    if constexpr (MODE == MODE_DIRECT_OBS) {
        if (active) {
            if (share) {
                RowSink o;
                o.row = grow; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
                emit_row_shared(v, c, sh, 0, o, ib);
            } else if (fast) {
                fill_obs_fast(v, c, 0, grow, ib);
            } else {
                fill_obs_slow(v, c, 0, grow, ib);
            }
        }
    } else {
        // PPO's buffer.obs record of agent rec_agent (Params::rec_obs, N = 2)
        RecRows rec{nullptr, 0, false};
        if constexpr (REC)
            rec = RecRows{(char *)(c.p->rec_obs + w0 * (int64_t)OW), c.p->rec_agent, c.p->rec_only != 0};
        else if (mirror_sim)
            rec = RecRows{(char *)(c.p->c.obs + w0 * N * (int64_t)OW), 0, false, true};
        if (active && !fast) {
            if (!(rec.base && rec.only && k == rec.agent)) fill_obs_slow(v, c, 0, grow, ib);
            if (REC && rec.base && k == rec.agent) fill_obs_slow(v, c, 0, c.p->rec_obs + w * (int64_t)OW, ib);
            if (!REC && mirror_sim) fill_obs_slow(v, c, 0, c.p->c.obs + (w * N + k) * (int64_t)OW, ib);
        }
        obs_phases<N, MODE, T>(v, c, sh, share, fast, tile, obs, w0 * N, lane, ib, rec);
        if (REC && T::QW < OW / 4) {
            // the record rows' zero tail (pieces QW .. OW/4 - 1), which the
            // passes do not write (the sim's own rows keep theirs from construction)
            constexpr int ZP = OW / 4 - T::QW, TOT = (WAVE / N) * ZP;
            const vf4 z = {0.f, 0.f, 0.f, 0.f};
            const uint64_t staged = __ballot(fast);  // rows that went through the tile
#pragma unroll
            for (int i = 0; i < (TOT + WAVE - 1) / WAVE; i++) {
                const int f = i * WAVE + lane, wl = f / ZP;
                if (f < TOT && ((staged >> (wl * N + rec.agent)) & 1ull))
                    row_store<BB_REC_AUX>(rec.base, (uint32_t)(wl * OW * 4 + (T::QW + f % ZP) * 16), z);
            }
        }
    }
}

// One lane per agent: lane = (w - w0) * N + k (blk: the wave's world group).
template <int N, int MODE, bool LINES, bool REC = false>
__device__ __forceinline__ void step_agent_lanes(const Params &p, float *tile, int blk, int lane)
{
    using T = StepTile<N, LINES>;
    const int k = lane % N;
    const int64_t w0 = (int64_t)blk * (WAVE / N);
    const int64_t w = w0 + lane / N;
    const bool active = w < p.num_worlds;  // uniform over the N lanes of a world
    const LaneAgents<N, MODE> ag{k, &p};

    World<N> s;
    Ctx c = make_ctx(p, w, k == 0);
    World<N> v;  // the world with this lane's agent in slot 0
    trace_point<MODE>(p, 0);
    // The event-only words as loaded (store only on change, see Orig) wait
    // in the observation tile, which is free until the observation pass:
    // registers stay with the systems.
    static_assert(sizeof(LaneOrig) / 4 * WAVE <= T::FLOATS, "parked words fit the tile");
    if (active) {
        load_world(s, p, w);
        {
            Orig<N> o;
            capture(o, s);
            LaneOrig x;
            x.world = world_orig(o);
            x.agent = pick_by<N>(k, [&](int j) { return o.ag[j]; });
            park_words(tile, lane, x);
        }
    }
    if (active) {
        if constexpr (MODE == MODE_SKIP) step_world_pre_obs(s, c, ag, p.diag_skip, p.diag_dup);
        else if constexpr (MODE != MODE_IO && MODE != MODE_IO_OBS) step_world_pre_obs(s, c, ag);
    }
    trace_point<MODE>(p, 7);
    trace_resets<MODE>(p, active, s);
    if (active) {
        agent_view(s, v, k);
        // reward + state columns first, so their stores drain while the
        // observation row is built
        if constexpr (MODE != MODE_IO && MODE != MODE_IO_OBS) sys_reward_agent(v, 0, AGENT0_ID + k);
        const LaneOrig x = unpark_words<LaneOrig>(tile, lane);
        store_world_agent<N, BB_COL_AUX>(v, p, w * N + k, 0, &x.agent);
        if (k == 0) {
            Orig<N> o;
            set_world_orig(o, x.world);
            store_world_shared<N, BB_COL_AUX>(s, p, w, &o);
        }
    }
    trace_point<MODE>(p, 8);
    if constexpr (MODE == MODE_IO || MODE == MODE_NO_OBS) return;

    const int32_t ib = active ? inbounder_id(s) : -1;
    const bool share = active && obs_sharable(s);
    agent_lane_obs<N, MODE, T, REC>(v, c, ib, share, k, lane, w0, w, active, tile, p.c.obs);
    trace_point<MODE>(p, 9);
}

// Pass PHASE of the observation rows of a wave that only writes rows (the
// observation wave of k_rollout_split): its own tile, wave-local ordering.
// mirror (wave-uniform, optional): every row also into this [W][N][OBSW] base.
template <int N, int PHASE, class T = StepTile<N, false>>
__device__ __forceinline__ void obs_pass_wave(const World<N> &v, const Ctx &c, int32_t ib, bool share, int k, int lane,
                                              int64_t w0, int64_t w, bool active, float *tile, float *obs,
                                              float *mirror = nullptr)
{
    constexpr int OW = obs_width(N);
    SharedObs<N> sh;
    lane_shared_obs(v, c, active, sh);
    const bool fast = active && canonical_slots(v, 0);
    // rows the tile does not carry are written whole by the first pass's wave
    if (PHASE == 0 && active && !fast) {
        fill_obs_slow(v, c, 0, obs + (w * N + k) * (int64_t)OW, ib);
        if (mirror) fill_obs_slow(v, c, 0, mirror + (w * N + k) * (int64_t)OW, ib);
    }
    if (fast) emit_phase<N, T, PHASE>(v, c, sh, share, tile + lane * T::RS, ib);
    wave_sync();
    constexpr int Q0 = PHASE * T::QP, QN = (T::QW - Q0 < T::QP) ? T::QW - Q0 : T::QP;
    constexpr int QZ = T::QU - Q0 < 0 ? 0 : (T::QU - Q0 < QN ? T::QU - Q0 : QN);
    const RecRows rec{mirror ? (char *)(mirror + w0 * N * (int64_t)OW) : nullptr, 0, false, true};
    flush_tile<N, T::QP, T::RS, Q0, QN, 1, QZ, T::AUX>(tile, obs, w0 * N, __ballot(fast), lane, rec);
}

// ------------------------------------------------------------------ rollout
// K steps in one launch (agent lanes, N = 2): the world stays in registers
// from the first load to the last store, so a step moves only its action
// rows in and its observation rows, rewards and done flags out -- exactly
// what K launches of k_step would leave in those buffers (bb_rollout).
// Step t+1's action rows are loaded before step t's stores are issued, so
// the stores of one step drain while the next one's systems run.
template <int N>
struct FusedRollout {
    static constexpr bool value = Lanes<N>::LPW == N && !Lanes<N>::SHARED;
};

// STORE (RolloutArgs::store_state): every step also stores the state columns
// (bb_step_n_staged's resident loop; a template parameter so the rollouts'
// code is untouched by it).
// (The resident loop keeps the rollout's whole-line row tile although its rows
// stay cache-resident: k_step's 2 x 13-piece rows measured slower there,
// 65 536 x 2 15.76 -> 18.48 us per step, 32 768 8.76 -> 10.04;
// profiles/r05/aq_steptile_sweep.txt; two whole lines then the rest of the
// used row -- one partial line per row, no zero tail -- 15.76 -> 16.96,
// aw_linetile_sweep.txt.  It stores every state column every
// step: the event-only words parked in LDS so as to store those columns only
// when changed, as k_step does, measured slower too, 65 536 x 2 15.76 ->
// 17.07, 262 144 59.8 -> 65.4; profiles/r05/at_event_orig_sweep.txt.)
template <int N, bool STORE>
__device__ __forceinline__ void rollout_agent_lanes(const Params &p, const RolloutArgs &r, float *tile, int blk,
                                                    int lane)
{
    using T = RolloutTile<N>;
    static_assert(6 * WAVE <= T::FLOATS, "the tile parks the lanes' staged action rows");
    const int64_t w0 = (int64_t)blk * (WAVE / N);
    const int64_t w = w0 + lane / N;
    const bool active = w < p.num_worlds;  // uniform over the N lanes of a world
    const int64_t rows = p.num_worlds * N;  // [W][N] rows per step

    // Between steps only the lane's view of the world is live (agent k in
    // slot 0); each step rebuilds the creation-order world from it, so the
    // systems' and the observation pass's register sets never overlap.
    World<N> v;
    uint32_t a_next[6 * N];
    if (active) {
        World<N> s;
        load_world(s, p, w);
        agent_view(s, v, lane % N);
        load_words<6 * N>(r.actions, w, a_next);
    }
    const double *erf_tab = erf_table_lds();
    // Everything loaded so far has arrived before the loop: no register
    // enters it with a load pending (which would make the compiler wait for
    // the vector-memory counter inside every step).
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    for (int t = 0; t < r.steps; t++) {
        // Opaque per-step copies of the lane and world index: what derives
        // from them (column addresses, agent ids, the tile flush's per-piece
        // offsets) is recomputed each step instead of being hoisted out of the
        // loop (or shared with the load before it) and held in registers --
        // or spilled -- across it.  A spill reload is a memory load, and one
        // issued after a step's stores waits for all of them.
        int lane_t = lane;
        int64_t w_t = w;
        __asm__ volatile("" : "+v"(lane_t));
        __asm__ volatile("" : "+v"(w_t));
        const int k = lane_t % N;
        const int64_t row = w_t * N + k;
        Ctx c = make_ctx(p, w_t, k == 0);
        c.erf_tab = erf_tab;
        const LaneAgents<N, MODE_FULL> ag{k, &p};
        int32_t *act_t = r.actions + (int64_t)t * rows * 6;
        uint32_t *park = (uint32_t *)tile + lane_t;  // word q at park[q * WAVE]: idle until the observation pass
        int32_t ib = -1;
        bool share = false;
        if (active) {
            World<N> s;
            agent_view<N, true>(v, s, k);
#pragma unroll
            for (int i = 0; i < N; i++)
#pragma unroll
                for (int q = 0; q < 6; q++) s.act[i][q] = (int32_t)a_next[6 * i + q];
#pragma unroll
            for (int q = 0; q < 6; q++) park[q * WAVE] = (uint32_t)pick_by<N>(k, [&](int j) { return s.act[j][q]; });
            // (unconditional -- the last step re-reads its own rows -- so that
            // every path through the loop has the same loads in flight)
            load_words<6 * N>(t + 1 < r.steps ? act_t + rows * 6 : act_t, w_t, a_next);
            step_world_pre_obs(s, c, ag);
            // Retire the prefetch here, before this step's stores are issued:
            // waiting for it then waits only for what was issued before it
            // (the previous step's stores, drained during these systems).  At
            // the top of the next step the rows are already in registers.
#pragma unroll
            for (int q = 0; q < 6 * N; q++) __asm__ volatile("" : "+v"(a_next[q]));
            ib = inbounder_id(s);
            share = obs_sharable(s);
            agent_view(s, v, k);
            sys_reward_agent(v, 0, AGENT0_ID + k);
            if constexpr (STORE) {
                // the columns of step t as k_step stores them: the action row
                // (overrides included) into the staged rows, reward and done
                // into the sim's columns (r.reward / r.done here)
                Params ps = p;
                ps.c.action = act_t;
                store_world_agent<N>(v, ps, row, 0);
                if (k == 0) store_world_shared<N>(v, p, w_t);
            } else {
                r.reward[(int64_t)t * r.rd_step + row] = v.rew[0];
                r.done[(int64_t)t * r.rd_step + row] = v.done[0];
                // the defence AI's overrides go back into the staged rows
                bool changed = false;
#pragma unroll
                for (int q = 0; q < 6; q++) changed |= (uint32_t)v.act[0][q] != park[q * WAVE];
                if (changed) {
                    uint32_t a[6];
#pragma unroll
                    for (int q = 0; q < 6; q++) a[q] = (uint32_t)v.act[0][q];
                    store_words<6>(act_t, row, a);
                }
            }
        }
        __syncthreads();  // parked rows read before the tile is rewritten
        // (the last step of a recorded rollout: the rows into the sim's tensor too)
        agent_lane_obs<N, MODE_FULL, T>(v, c, ib, share, k, lane_t, w0, w_t, active, tile,
                                        r.obs + (int64_t)t * r.obs_step,
                                        t + 1 == r.steps && r.obs_step != 0);
        __syncthreads();  // the tile is rewritten by the next step
    }
    if (!STORE && active && r.steps > 0) {  // the simulator's own columns: state after the last step
        int64_t w_s = w;
        __asm__ volatile("" : "+v"(w_s));
        const int k = lane % N;
        store_world_agent(v, p, w_s * N + k, 0);
        if (k == 0) store_world_shared(v, p, w_s);  // world fields are not permuted in a view
    }
    if (STORE && active && r.steps > 0) {
        // the last step's action rows (overrides included) into the sim's
        // action tensor, as bb_step_n_staged leaves it (no copy launch after
        // the kernel): read back from the staged rows this lane stored last
        // (after the loop: nothing of the step waits on this load)
        int64_t w_s = w;
        __asm__ volatile("" : "+v"(w_s));
        const int64_t row = w_s * N + lane % N;
        uint32_t a[6];
        load_words<6>(r.actions + (int64_t)(r.steps - 1) * rows * 6, row, a);
        store_words<6>(p.c.action, row, a);
    }
}

// MINW: waves per SIMD the register budget is sized for.  2 (256 registers)
// spills the step loop's state (140 B of scratch per lane, reloaded on the
// chain every step); 1 gives the wave the SIMD's whole file (VGPRs + AGPRs,
// no scratch) and is taken while the grid is at most one wave per SIMD.
// G > 1: workgroups of G waves, kept in step by the loop's two barriers per
// step (not launched: G = 4 measured slower, 65 536 worlds 15.6-16.1 -> 16.6
// us per step, profiles/r05/ag_rollout_g_ab.txt).
template <int N, int MINW = 2, int G = 1, bool STORE = false>
__global__ __launch_bounds__(WAVE * G, MINW) void k_rollout(const Params p, const RolloutArgs r)
{
    if constexpr (FusedRollout<N>::value) {
        constexpr int TF = RolloutTile<N>::FLOATS;
        __shared__ float4 tile4[G * TF / 4];
        const int wave = G == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE);
        rollout_agent_lanes<N, STORE>(p, r, (float *)tile4 + wave * TF, (int)blockIdx.x * G + wave,
                                      (int)(threadIdx.x % WAVE));
    }
}

// K-step rollout over two waves per 32 worlds (C2-sized grids): the sim
// wave S runs rollout_agent_lanes' step loop up to the reward / done records
// and hands each lane's view of the world to the observation wave O through
// LDS; O writes step t's observation rows while S runs the systems of step
// t + 1.  Per step, with A / B the two workgroup barriers:
//   S: systems(t), records(t)  A  view(t) -> LDS  B
//   O:                         A                  B  LDS -> view(t), rows(t)
// A: O has read view(t-1) (the buffer is free); B: view(t) is in LDS.  The
// step's period is max(S's systems, O's rows) instead of their sum.  The rows
// are emitted by the same pass code on the same view: bit-identical to
// k_rollout.
template <int N>
struct SplitView {
    static constexpr int WORDS = (int)(sizeof(World<N>) / 4) + 2;  // the view, inbounder id, obs_sharable
    uint32_t w[WORDS][WAVE];  // word-major: word i of lane l at w[i][l]
};

template <int N, bool STORE>
__device__ __forceinline__ void split_sim_wave(const Params &p, const RolloutArgs &r, SplitView<N> &view,
                                               uint32_t *park_base)
{
    const int lane = (int)threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * (WAVE / N);
    const int64_t w = w0 + lane / N;
    const bool active = w < p.num_worlds;
    const int64_t rows = p.num_worlds * N;
    World<N> v;
    uint32_t a_next[6 * N];
    if (active) {
        World<N> s;
        load_world(s, p, w);
        agent_view(s, v, lane % N);
        load_words<6 * N>(r.actions, w, a_next);
    }
    const double *erf_tab = erf_table_lds();
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    for (int t = 0; t < r.steps; t++) {
        int lane_t = lane;
        int64_t w_t = w;
        __asm__ volatile("" : "+v"(lane_t));
        __asm__ volatile("" : "+v"(w_t));
        const int k = lane_t % N;
        const int64_t row = w_t * N + k;
        Ctx c = make_ctx(p, w_t, k == 0);
        c.erf_tab = erf_tab;
        const LaneAgents<N, MODE_FULL> ag{k, &p};
        int32_t *act_t = r.actions + (int64_t)t * rows * 6;
        uint32_t *park = park_base + lane_t;
        int32_t ib = -1;
        bool share = false;
        if (active) {
            World<N> s;
            agent_view<N, true>(v, s, k);
#pragma unroll
            for (int i = 0; i < N; i++)
#pragma unroll
                for (int q = 0; q < 6; q++) s.act[i][q] = (int32_t)a_next[6 * i + q];
#pragma unroll
            for (int q = 0; q < 6; q++) park[q * WAVE] = (uint32_t)pick_by<N>(k, [&](int j) { return s.act[j][q]; });
            load_words<6 * N>(t + 1 < r.steps ? act_t + rows * 6 : act_t, w_t, a_next);
            step_world_pre_obs(s, c, ag);
#pragma unroll
            for (int q = 0; q < 6 * N; q++) __asm__ volatile("" : "+v"(a_next[q]));
            ib = inbounder_id(s);
            share = obs_sharable(s);
            agent_view(s, v, k);
            sys_reward_agent(v, 0, AGENT0_ID + k);
            if constexpr (STORE) {  // as in rollout_agent_lanes
                Params ps = p;
                ps.c.action = act_t;
                store_world_agent<N>(v, ps, row, 0);
                if (k == 0) store_world_shared<N>(v, p, w_t);
            } else {
                r.reward[(int64_t)t * r.rd_step + row] = v.rew[0];
                r.done[(int64_t)t * r.rd_step + row] = v.done[0];
                bool changed = false;
#pragma unroll
                for (int q = 0; q < 6; q++) changed |= (uint32_t)v.act[0][q] != park[q * WAVE];
                if (changed) {
                    uint32_t a[6];
#pragma unroll
                    for (int q = 0; q < 6; q++) a[q] = (uint32_t)v.act[0][q];
                    store_words<6>(act_t, row, a);
                }
            }
        }
        lds_barrier();  // A: the observation wave has read view(t-1)
        {
            uint32_t u[SplitView<N>::WORDS];
            __builtin_memcpy(u, &v, sizeof(World<N>));
            u[SplitView<N>::WORDS - 2] = (uint32_t)ib;
            u[SplitView<N>::WORDS - 1] = share ? 1u : 0u;
#pragma unroll
            for (int i = 0; i < SplitView<N>::WORDS; i++) view.w[i][lane_t] = u[i];
        }
        lds_barrier();  // B: view(t) is in LDS
    }
    if (!STORE && active && r.steps > 0) {  // the simulator's own columns: state after the last step
        int64_t w_s = w;
        __asm__ volatile("" : "+v"(w_s));
        const int k = lane % N;
        store_world_agent(v, p, w_s * N + k, 0);
        if (k == 0) store_world_shared(v, p, w_s);
    }
    if (STORE && active && r.steps > 0) {  // the last step's action rows into the sim's action tensor
        int64_t w_s = w;
        __asm__ volatile("" : "+v"(w_s));
        const int64_t row = w_s * N + lane % N;
        uint32_t a[6];
        load_words<6>(r.actions + (int64_t)(r.steps - 1) * rows * 6, row, a);
        store_words<6>(p.c.action, row, a);
    }
}

template <int N, class T>
__device__ __forceinline__ void split_obs_wave(const Params &p, const RolloutArgs &r, const SplitView<N> &view,
                                               float *tile)
{
    const int lane = (int)threadIdx.x % WAVE;
    const int64_t w0 = (int64_t)blockIdx.x * (WAVE / N);
    for (int t = 0; t < r.steps; t++) {
        int lane_t = lane;
        __asm__ volatile("" : "+v"(lane_t));
        const int64_t w = w0 + lane_t / N;
        const bool active = w < p.num_worlds;
        const int k = lane_t % N;
        lds_barrier();  // A
        lds_barrier();  // B
        World<N> v;
        uint32_t u[SplitView<N>::WORDS];
#pragma unroll
        for (int i = 0; i < SplitView<N>::WORDS; i++) u[i] = view.w[i][lane_t];
        __builtin_memcpy(&v, u, sizeof(World<N>));
        const int32_t ib = (int32_t)u[SplitView<N>::WORDS - 2];
        const bool share = u[SplitView<N>::WORDS - 1] != 0u;
        const Ctx c = make_ctx(p, w, k == 0);
        float *obs = r.obs + (int64_t)t * r.obs_step;
        // the last step of a recorded rollout: the rows into the sim's tensor too
        float *mirror = (t + 1 == r.steps && r.obs_step != 0) ? p.c.obs : nullptr;
        obs_pass_wave<N, 0, T>(v, c, ib, share, k, lane_t, w0, w, active, tile, obs, mirror);
        wave_sync();  // the tile is rewritten by the next pass
        if constexpr (T::PH > 1) {
            obs_pass_wave<N, 1, T>(v, c, ib, share, k, lane_t, w0, w, active, tile, obs, mirror);
            wave_sync();
        }
        static_assert(T::PH <= 2, "two row passes");
    }
}

template <int N, bool STORE = false>
__global__ __launch_bounds__(2 * WAVE, 1) void k_rollout_split(const Params p, const RolloutArgs r)
{
    if constexpr (FusedRollout<N>::value) {
        using T = RolloutTile<N>;
        __shared__ SplitView<N> view;
        __shared__ float4 tile4[T::FLOATS / 4];
        __shared__ uint32_t park[6 * WAVE];
        if (__builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE) == 0) split_sim_wave<N, STORE>(p, r, view, park);
        else split_obs_wave<N, T>(p, r, view, (float *)tile4);
    }
}

// ------------------------------------------------------------------ PPO rollout
// scripts/ppo.py:61-141 in one launch (bb_rollout_policy, N = 2): a workgroup
// of 1 + PW waves per 32 worlds (PW policy waves).  Wave S holds the worlds in
// registers for all K steps (rollout_agent_lanes' discipline); the policy
// waves P hold the network's B operands in registers (k_policy's) and own 16
// trainee rows each.  Per step k:
//   P: record the trainee's observation X (LDS) into obs_out[k], the network
//      on X (policy_layers / bucket_pass_spread, bit-identical to k_policy),
//      actions into LDS and act_out[k], log-prob and value;   -> barrier
//   S: the trainee's action from LDS (the other agent keeps what the sim left
//      in its action column), systems 1-17 and reward, reward / done of the
//      trainee into reward[k] / done[k], the trainee's next observation row
//      into X (and on the last step every row into the sim's tensor);  -> barrier
// then P's value pass over the final X gives next_value (ppo.py:136-137), and S
// stores every column of the worlds (the state after step K-1).
// Policy waves: one per 16-row M-tile (policy_layers1_split: both output
// halves of every product in the one wave, the LayerNorms on its own
// registers), so nothing inside the network crosses waves: a step has four
// workgroup barriers -- X's first half ready, its second half, the actions,
// X free.  (Until round 5 two waves per M-tile ran one output half each and
// exchanged accumulators for the LayerNorms: five more barriers per step,
// 8 192-world trace 4.56 us for the policy pass.)
// The waves of the PPO workgroup share nothing through global memory inside
// the loop, so their hand-offs are lds_barrier()s, which do not wait for the
// wave's outstanding global stores (a __syncthreads() release fence does:
// vmcnt(0) before every hand-off, ~1 us of write latency per step).
// PW policy waves per 32 worlds: 2 (one per M-tile) or 4 (two per M-tile,
// one output half each: policy_layers_half_split, accumulators exchanged
// through LDS for the LayerNorms, 5 more workgroup barriers per step, 8 rows
// per bucket pass).  launch_rollout_policy_t picks PW.
template <int PW>
struct PpoCfg {
    static constexpr int LAYER_BARS = PW == 4 ? 5 : 0;
    static constexpr int ROWS = 32 / PW;  // rows per policy wave's bucket pass
};
constexpr int PPO_XS = 132;  // LDS row stride of X (floats)
template <int PW>
struct PpoLds {
    float x[32][PPO_XS];
    int32_t act[32][6];
    float norm[2][POL_IN];
    float ptile[2][16][33];   // each M-tile's hidden activations, then (2 waves) logits + value
    float ltile[PW == 4 ? 2 : 1][16][33];  // (4 waves) logits + value of each M-tile
    HalfExchange ex[PW == 4 ? 2 : 1];
    BucketLds<32 / PW> bucket[PW];
    double erf[ERF_WORDS];
};

// RowSink into an LDS row (X)
struct LdsRowSink {
    float *row;
    float b0, b1, b2, b3;
    int idx;
    __device__ void put(float v)
    {
        switch (idx & 3) {
        case 0: b0 = v; break;
        case 1: b1 = v; break;
        case 2: b2 = v; break;
        default: *(float4 *)(row + (idx & ~3)) = make_float4(b0, b1, b2, v); break;
        }
        idx++;
    }
    __device__ void put3(F3 v) { put(v.x); put(v.y); put(v.z); }
    __device__ void put4(Q4 q) { put(q.w); put(q.x); put(q.y); put(q.z); }
    __device__ void finish() { while (idx & 3) put(0.f); }
};

// The trainee's observation row in two hand-offs: pass P holds row floats i
// with ((i >> 4) & 1) == P (for every lane group q of layer 1 the chain steps
// j = 16P .. 16P + 15), written at their own positions of X.  With ROLE >= 0
// the world's two lanes share a pass: the trainee's lane (ROLE 0) writes the
// floats with ((i >> 3) & 1) == 0, the other lane (ROLE 1, the trainee's row
// emitted from its own view, observer slot 1) the rest.
template <int P, int ROLE>
struct XPassSink {
    float *row;
    float b0, b1, b2, b3;
    int idx;
    __device__ void put(float v)
    {
        if (((idx >> 4) & 1) == P && (ROLE < 0 || ((idx >> 3) & 1) == ROLE)) {
            switch (idx & 3) {
            case 0: b0 = v; break;
            case 1: b1 = v; break;
            case 2: b2 = v; break;
            default: *(float4 *)(row + (idx & ~3)) = make_float4(b0, b1, b2, v); break;
            }
        }
        idx++;
    }
    __device__ void put3(F3 v) { put(v.x); put(v.y); put(v.z); }
    __device__ void put4(Q4 q) { put(q.w); put(q.x); put(q.y); put(q.z); }
    __device__ void finish() { while (idx & 3) put(0.f); }
};

// Pass P of the trainee's row of the lane's world into X (row xr).  split:
// both lanes of the world emit (shared intrinsic blocks, canonical slots);
// otherwise the trainee's lane emits the pass alone (a non-canonical world's
// whole row in pass 0, by the runtime-indexed sink).
template <int P>
__device__ __forceinline__ void ppo_x_pass(const World<2> &v, const Ctx &c, const SharedObs<2> &sh, bool active,
                                           bool is_trainee, bool split, bool fast, float *xr, int32_t ib)
{
    if (!active) return;
    if (split) {
        if (is_trainee) {
            XPassSink<P, 0> o;
            o.row = xr; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
            emit_row_shared(v, c, sh, 0, o, ib);
        } else {
            XPassSink<P, 1> o;
            o.row = xr; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
            emit_row_shared(v, c, sh, 1, o, ib);
        }
    } else if (is_trainee) {
        if (fast) {
            XPassSink<P, -1> o;
            o.row = xr; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
            emit_row_fast(v, c, 0, o, ib);
        } else if (P == 0) {
            fill_obs_slow(v, c, 0, xr, ib);
        }
    }
}

template <int N, int PW>
__device__ __forceinline__ void ppo_sim_wave(const Params &p, const PolicyRolloutArgs &r, PpoLds<PW> &L, float *tile)
{
    static_assert(N == 2, "the reference's 2-agent game");
    const int lane = threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * (WAVE / N);
    const int64_t w = w0 + lane / N;
    const int wl = lane / N;
    const bool active = w < p.num_worlds;
    const int trainee = r.trainee;
    World<N> v;
    if (active) {
        World<N> s;
        load_world(s, p, w);
        agent_view(s, v, lane % N);
    }
    {
        const double *g = &bbm::ERF_TAYLOR[0][0];
#pragma unroll
        for (int j = 0; j < (ERF_WORDS + WAVE - 1) / WAVE; j++) {
            const int i = j * WAVE + lane;
            if (i < ERF_WORDS) L.erf[i] = g[i];
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no load pending into the loop
    lds_barrier();  // setup: X holds the trainee rows of step 0, the erf table is in LDS
    lds_barrier();  // (step 0's two row hand-offs: X is complete already)
    lds_barrier();
    for (int t = 0; t < r.steps; t++) {
        int lane_t = lane;
        int64_t w_t = w;
        __asm__ volatile("" : "+v"(lane_t));
        __asm__ volatile("" : "+v"(w_t));
        const int k = lane_t % N;
        Ctx c = make_ctx(p, w_t, k == 0);
        c.erf_tab = L.erf;
        const LaneAgents<N, MODE_FULL> ag{k, &p};
        for (int b = 0; b < PpoCfg<PW>::LAYER_BARS; b++) lds_barrier();  // (the policy pass's own barriers)
        lds_barrier();  // the policy's actions are in LDS
        int32_t ib = -1;
        bool share = false;
        if (active) {
            World<N> s;
            agent_view<N, true>(v, s, k);
            int32_t a[6];
#pragma unroll
            for (int q = 0; q < 6; q++) a[q] = L.act[wl][q];
#pragma unroll
            for (int i = 0; i < N; i++)
#pragma unroll
                for (int q = 0; q < 6; q++) s.act[i][q] = i == trainee ? a[q] : s.act[i][q];
            step_world_pre_obs(s, c, ag);
            ib = inbounder_id(s);
            share = obs_sharable(s);
            agent_view(s, v, k);
        }
        // the trainee's next observation row into X, in two hand-offs
        SharedObs<N> sh;
        lane_shared_obs(v, c, active, sh);
        const bool is_trainee = k == trainee;
        const bool fast = active && canonical_slots(v, 0);
        const bool split = share && fast;  // uniform over the world's two lanes
        if (active && split && !is_trainee) {
            // the trainee's direction / distance to this lane's agent, as the
            // trainee's lane computes them (lane_shared_obs: to = other - self)
            const F3 to = v.pos(0) - v.pos(1);
            const float l2 = len2(to);
            const float rr = 1.0f / bbm::sqrtf_(l2);
            sh.rdir[1][0] = l2 > 1e-6f ? to * rr : f3(0.f, 0.f, 0.f);
            sh.rlen[1][0] = bbm::sqrtf_(l2);
        }
        float *xr = L.x[wl];
        lds_barrier();  // X is free: the policy waves have recorded buffer.obs[t] from it
        ppo_x_pass<0>(v, c, sh, active, is_trainee, split, fast, xr, ib);
        wave_sync();
        lds_barrier();  // pass 0 of X: the policy waves start layer 1
        ppo_x_pass<1>(v, c, sh, active, is_trainee, split, fast, xr, ib);
        wave_sync();
        lds_barrier();  // X holds the observations after step t
        if (t + 1 == r.steps) {  // the sim's observation tensor: every row of the last step
            // (beside the policy waves' value pass, which reads X only)
            obs_pass_wave<N, 0>(v, c, ib, share, k, lane_t, w0, w_t, active, tile, p.c.obs);
            wave_sync();
            obs_pass_wave<N, 1>(v, c, ib, share, k, lane_t, w0, w_t, active, tile, p.c.obs);
        }
        // reward (read by nothing on the way to the next actions) while the
        // policy waves run the network on X
        if (active) {
            sys_reward_agent(v, 0, AGENT0_ID + k);
            if (k == trainee && r.reward) {
                r.reward[(int64_t)t * p.num_worlds + w_t] = v.rew[0];
                r.done[(int64_t)t * p.num_worlds + w_t] = v.done[0];
            }
        }
    }
    if (active && r.steps > 0) {  // the simulator's own columns: state after the last step
        int64_t w_s = w;
        __asm__ volatile("" : "+v"(w_s));
        const int k = lane % N;
        store_world_agent(v, p, w_s * N + k, 0);
        if (k == 0) store_world_shared(v, p, w_s);
    }
    for (int b = 0; b < PpoCfg<PW>::LAYER_BARS; b++) lds_barrier();  // (the next-value pass's barriers)
}

template <int PW>
__device__ __forceinline__ void ppo_policy_wave(const Params &p, const PolicyRolloutArgs &r, PpoLds<PW> &L, int pw)
{
    constexpr int RW = PpoCfg<PW>::ROWS;                              // this wave's rows (bucket pass, records)
    const int lane = threadIdx.x % WAVE, c = lane & 15, q = lane >> 4;
    const int64_t W = p.num_worlds;
    const int m = PW == 4 ? pw >> 1 : pw;             // M-tile
    const int h = PW == 4 ? pw & 1 : 0;               // (4 waves) column half
    const int r0 = 16 * m;                                    // first X row of the M-tile
    const int rh = RW * h;                                    // this wave's rows of the M-tile
    const int64_t row0 = (int64_t)blockIdx.x * 32 + r0;       // the M-tile's first world
    // network constants: norm by the lanes of the policy waves, B operands per lane
    for (int k = pw * WAVE + lane; k < POL_IN; k += PW * WAVE) {
        L.norm[0][k] = r.w.obs_mean[k];
        L.norm[1][k] = r.w.obs_inv[k];
    }
    PolicyRegs R;
    load_policy_regs(R, r.w, c, q);
    // X for step 0: this wave's trainee rows of the sim's observation tensor
    // (with their zero tail, which emit never writes)
    for (int i = lane; i < RW * 32; i += WAVE) {
        const int rr = r0 + rh + i / 32, qq = i % 32;
        const int64_t wg = (int64_t)blockIdx.x * 32 + rr;
        float4 v4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (wg < W) v4 = *(const float4 *)(p.c.obs + (wg * 2 + r.trainee) * (int64_t)obs_width(2) + 4 * qq);
        *(float4 *)&L.x[rr][4 * qq] = v4;
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    lds_barrier();  // setup
    PolicyArgs a{};
    a.rows = W;
    a.stochastic = r.stochastic;
    a.seed = r.seed;
    // the sampling uniforms of a step depend on (seed, step, row, bucket) only: each
    // step's is drawn while the sim wave runs the step before it
    BucketNoise<RW> noise;
    if (r.stochastic) bucket_noise<RW>(noise, r.seed, r.step0, row0 + rh, W, lane);
    for (int t = 0; t <= r.steps; t++) {
        const bool final_pass = t == r.steps;  // agent.evaluate(obs_): value only
        lds_barrier();  // pass 0 of X: the rows' first half
        auto mid = [&] {
            lds_barrier();  // the rows' second half
        };
        float (*lt)[33];
        if constexpr (PW == 4) {
            auto bar = [] { lds_barrier(); };
            policy_layers_half_split(&L.x[r0 + c][0], R, L.norm, L.ptile[m], L.ltile[m], L.ex[m], c, q, lane, h, mid,
                                     bar);
            lt = L.ltile[m];
        } else {
            policy_layers1_split(&L.x[r0 + c][0], R, L.norm, L.ptile[m], c, q, mid);
            lt = L.ptile[m];
        }
        a.step = r.step0 + (uint32_t)t;
        if (!final_pass) {
            a.act_out = r.act_out ? r.act_out + (int64_t)t * W * 6 : nullptr;
            a.log_prob = r.log_prob ? r.log_prob + (int64_t)t * W : nullptr;
            a.value = r.value ? r.value + (int64_t)t * W : nullptr;
            // the actions first (all the sim wave waits for), the log-probs
            // and the records behind the hand-off
            BucketHold<RW> hold;
            if (r.stochastic)
                bucket_pass_act<RW, true>(a, lt + rh, row0 + rh, lane, L.bucket[pw], L.act + r0 + rh, &noise, hold);
            else
                bucket_pass_act<RW, false>(a, lt + rh, row0 + rh, lane, L.bucket[pw], L.act + r0 + rh, nullptr, hold);
            pol_wave_sync();
            lds_barrier();  // actions in LDS
            bucket_pass_out<RW>(a, lt + rh, row0 + rh, lane, L.bucket[pw], hold);
            // while the sim wave steps: buffer.obs[t] = X (this wave's rows),
            // then the next step's sampling uniforms
            if (r.obs_out) {
                for (int i = lane; i < RW * 32; i += WAVE) {
                    const int rr = r0 + rh + i / 32, qq = i % 32;
                    const int64_t wg = (int64_t)blockIdx.x * 32 + rr;
                    if (wg < W)
                        *(float4 *)(r.obs_out + ((int64_t)t * W + wg) * POL_IN + 4 * qq) = *(const float4 *)&L.x[rr][4 * qq];
                }
            }
            if (r.stochastic && t + 1 < r.steps)
                bucket_noise<RW>(noise, r.seed, r.step0 + (uint32_t)(t + 1), row0 + rh, W, lane);
            lds_barrier();  // X is free (the sim wave rewrites it next)
        } else if (r.next_value && lane < RW && row0 + rh + lane < W) {
            r.next_value[row0 + rh + lane] = lt[rh + lane][POL_LOGITS];
        }
    }
}

// MINW: waves per SIMD the register budget is sized for -- 1 while the grid
// is one workgroup per CU (each of its 3 waves then has a SIMD to itself and
// the sim wave keeps its world without spills), 2 above
template <int N, int MINW, int PW>
__global__ __launch_bounds__(WAVE * (1 + PW), MINW) void k_rollout_policy(const Params p, const PolicyRolloutArgs r)
{
    if constexpr (N == 2 && FusedRollout<N>::value) {
        __shared__ PpoLds<PW> L;
        __shared__ float4 tile4[StepTile<N, false>::FLOATS / 4];
        const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE);
        if (wave == 0) ppo_sim_wave<N, PW>(p, r, L, (float *)tile4);
        else ppo_policy_wave<PW>(p, r, L, wave - 1);
    }
}

// ------------------------------------------------------------------ PPO step
// k_step_ppo<2>: one step of PPO's rollout loop with the trainee's policy pass
// fused behind it (bb_rollout_policy above 16 384 worlds; scripts/ppo.py:65-134
// over scripts/env.py:126-170).  A wave steps its 32 worlds exactly as
// k_step<2> does (agent lanes, the world in registers), then the policy of
// step k + 1 runs on the trainee's rows while they are in LDS: no second
// launch, and the 512 bytes of each trainee row are never read back from HBM.
//
// Row passes split by the policy's layer-1 chain order.  Layer 1 is the
// k-ordered MFMA chain of policy_layers: step j (0..31) feeds lane group q with
// observation float 32q + j.  Pass P of the rows holds the floats with
// ((i >> 4) & 1) == P -- for every q the steps j = 16P .. 16P + 15 -- at tile
// slot (i >> 5) * 16 + (i & 15): pass 0 slots 0..55 (floats 96..103 of q = 3
// included; 104..127 are the row's zero tail), pass 1 slots 0..47.  After a
// pass is in the tile, the wave runs that pass's 16 chain steps for its two
// 16-row M-tiles of trainee rows (the same operands in the same order as
// every other policy kernel: bit-identical), then stores the pass's pieces.
// The network's weights sit in LDS once per workgroup of WPG waves
// (PolicyLdsWeights, 32.6 KB); each wave's tile (64 rows x 60 floats, 15 KB)
// takes the LayerNorm / bucket-pass exchanges after the last pass.
constexpr int PPS_RS = 60;  // tile row stride (floats): 14 pieces + 1, == 4 mod 8 dwords
// buffer.obs rows (half lines per pass): write-through -- measured at 65 536
// worlds 39.3 us per step vs 40.5 nt, 42.3 plain (profiles/r05/c_rec_policy_ab.txt)
#ifndef BB_PPS_REC_AUX
#define BB_PPS_REC_AUX 16
#endif
constexpr int PPS_TILE = WAVE * PPS_RS;

template <int WPG>
struct PpoStepLds {
    PolicyLdsWeights wt;
    float tile[WPG][PPS_TILE];
};

// Floats of pass P of a row into its tile row (compile-time indices: straight
// float4 LDS writes of the pass's pieces, the other floats never computed).
template <int P>
struct PassSink {
    float *row;
    float b0, b1, b2, b3;
    int idx;
    __device__ void put(float v)
    {
        if (((idx >> 4) & 1) == P && idx < 4 * PhasedTile<2>::QU) {
            switch (idx & 3) {
            case 0: b0 = v; break;
            case 1: b1 = v; break;
            case 2: b2 = v; break;
            default: *(float4 *)(row + ((idx >> 5) << 4) + (idx & 12)) = make_float4(b0, b1, b2, v); break;
            }
        }
        idx++;
    }
    __device__ void put3(F3 v) { put(v.x); put(v.y); put(v.z); }
    __device__ void put4(Q4 q) { put(q.w); put(q.x); put(q.y); put(q.z); }
    __device__ void finish() { while (idx & 3) put(0.f); }
};
// The same for the rows of non-canonical team layouts (runtime indices).
template <int P>
struct PassSlowSink {
    float *row;
    int idx;
    __device__ void put(float v)
    {
        if (idx < 4 * PhasedTile<2>::QU && ((idx >> 4) & 1) == P) row[((idx >> 5) << 4) + (idx & 15)] = v;
        idx++;
    }
    __device__ void put3(F3 v) { put(v.x); put(v.y); put(v.z); }
    __device__ void put4(Q4 q) { put(q.w); put(q.x); put(q.y); put(q.z); }
};

// Layer-1 chain steps 16P .. 16P + 15 of the wave's two M-tiles of trainee
// rows (row m = 16 mt + c is world w0 + m; its tile row 2m + trainee).
template <int P>
__device__ __forceinline__ void ppo_layer1_pass(const float *tile, const PolicyLdsWeights &L, f32x4 (&acc)[2][2],
                                                int trainee, int c, int q)
{
    constexpr int QD = P == 0 ? 2 : 0;  // float4 groups of lane group q = 3 holding row values
    const int ng = q < 3 ? 4 : QD;
    const float *r0 = tile + (2 * c + trainee) * PPS_RS + 16 * q;
    const float *r1 = r0 + 32 * PPS_RS;
#pragma unroll
    for (int v = 0; v < 4; v++) {
        const float4 m4 = *(const float4 *)&L.norm[0][32 * q + 16 * P + 4 * v];
        const float4 i4 = *(const float4 *)&L.norm[1][32 * q + 16 * P + 4 * v];
        const float4 b0 = *(const float4 *)&L.w1[q][c][16 * P + 4 * v];
        const float4 b1 = *(const float4 *)&L.w1[q][16 + c][16 * P + 4 * v];
        // lanes past their row values read their row's first piece (a valid
        // address) and feed the zero tail
        const bool has = v < ng;
        const int o = has ? 4 * v : 0;
        float4 x0 = *(const float4 *)(r0 + o), x1 = *(const float4 *)(r1 + o);
        if (!has) x0 = x1 = make_float4(0.f, 0.f, 0.f, 0.f);
        const float nm[4] = {m4.x, m4.y, m4.z, m4.w}, ni[4] = {i4.x, i4.y, i4.z, i4.w};
        const float w0[4] = {b0.x, b0.y, b0.z, b0.w}, w1[4] = {b1.x, b1.y, b1.z, b1.w};
        const float xa[4] = {x0.x, x0.y, x0.z, x0.w}, xb[4] = {x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const float ya = pol_clamp((xa[e] - nm[e]) * ni[e]);
            const float yb = pol_clamp((xb[e] - nm[e]) * ni[e]);
            acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(ya, w0[e], acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ya, w1[e], acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(yb, w0[e], acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(yb, w1[e], acc[1][1], 0, 0, 0);
        }
    }
}

// Stores of pass P: tile piece t of row r is row piece 8 (t >> 2) + 4P + (t & 3).
// Sim rows (ALL, the last step: every row): the pass's NS pieces of the 64
// rows.  Before the last step no sim row is stored: the trainee's goes to
// buffer.obs only, and the other agent's is read by nobody before the last
// step rewrites it (no opponent policy on this path; 27 MB per step at 65 536
// worlds).  Record rows (buffer.obs, the trainee's): 16 pieces per pass, the
// zero tail included, at rec + m * 512.  Rows of worlds past the grid's end
// (bit clear in `live`) store nothing.
template <int P, bool ALL>
__device__ __forceinline__ void ppo_flush_pass(const float *tile, char *obs, char *rec, uint64_t live, int trainee,
                                               int lane)
{
    constexpr int NS = P == 0 ? 14 : 12;
    constexpr int SIT = NS;  // store instructions: 64 rows x NS pieces
    constexpr int OWB = 128 * 4;
    if constexpr (ALL) {
        vf4 v[SIT];
        uint32_t off[SIT];
        bool ok[SIT];
#pragma unroll
        for (int i = 0; i < SIT; i++) {
            const int f = i * WAVE + lane, r = f / NS, t = f - r * NS;
            ok[i] = (live >> r) & 1ull;
            off[i] = (uint32_t)(r * OWB + (8 * (t >> 2) + 4 * P + (t & 3)) * 16);
            v[i] = *(const vf4 *)(tile + r * PPS_RS + 4 * t);
        }
#pragma unroll
        for (int i = 0; i < SIT; i++)
            if (ok[i]) row_store<BB_STEP_AUX>(obs, off[i], v[i]);
    }
    if (rec) {  // wave-uniform
        constexpr int RIT = (WAVE / 2) * 16 / WAVE;  // 8
        vf4 v[RIT];
        uint32_t off[RIT];
        bool ok[RIT];
#pragma unroll
        for (int i = 0; i < RIT; i++) {
            const int f = i * WAVE + lane, m = f >> 4, t = f & 15;
            const int r = 2 * m + trainee;
            ok[i] = (live >> r) & 1ull;
            off[i] = (uint32_t)(m * OWB + (8 * (t >> 2) + 4 * P + (t & 3)) * 16);
            v[i] = t < NS ? *(const vf4 *)(tile + r * PPS_RS + 4 * t) : vf4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int i = 0; i < RIT; i++)
            if (ok[i]) row_store<BB_PPS_REC_AUX>(rec, off[i], v[i]);
    }
}

template <int P>
__device__ __forceinline__ void ppo_emit_pass(const World<2> &v, const Ctx &c, const SharedObs<2> &sh, bool active,
                                              bool fast, bool share, float *trow, int32_t ib)
{
    if (!active) return;
    if (fast) {
        PassSink<P> o;
        o.row = trow; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
        if (share) emit_row_shared(v, c, sh, 0, o, ib);
        else emit_row_fast(v, c, 0, o, ib);
    } else {
        PassSlowSink<P> o;
        o.row = trow; o.idx = 0;
        emit_row_slow(v, c, 0, o, ib);
    }
}

// Step k of a k_rollout_ppo launch: a0 holds step 0's outputs (reward /
// done [k], buffer.obs / actions / log_probs / values [k + 1]); the last step
// writes next_value (a0.value_last) and no buffer entries of step k + 1.
__device__ __forceinline__ PpoStepArgs ppo_loop_args(const PpoStepArgs &a0, int32_t k, int32_t steps, int64_t W)
{
    PpoStepArgs a = a0;
    const int64_t o = (int64_t)k * W;
    if (a.reward) {
        a.reward += o;
        a.done += o;
    }
    a.step = a0.step + (uint32_t)k;
    a.last = k + 1 == steps ? 1 : 0;
    if (a.last) {
        a.obs_rec = nullptr;
        a.act_out = nullptr;
        a.log_prob = nullptr;
        a.value = a0.value_last;
    } else {
        if (a.obs_rec) a.obs_rec += o * POL_IN;
        if (a.act_out) a.act_out += o * 6;
        if (a.log_prob) a.log_prob += o;
        if (a.value) a.value += o;
    }
    return a;
}

// LOOP: a step of k_rollout_ppo's loop (the weights are in LDS already; no
// workgroup barrier, the waves run their worlds' steps independently).
template <int WPG, bool LAST, bool LOOP = false>
__device__ __forceinline__ void ppo_step_wave(const Params &p, const PpoStepArgs &a, PpoStepLds<WPG> &S, int blk,
                                              int wave, int lane)
{
    constexpr int N = 2;
    float *tile = S.tile[wave];
    const int k = lane % N;
    const int64_t w0 = ((int64_t)blk * WPG + wave) * (WAVE / N);
    const int64_t w = w0 + lane / N;
    const bool active = w < p.num_worlds;  // uniform over the N lanes of a world
    const int trainee = a.trainee;
    const LaneAgents<N, MODE_FULL> ag{k, &p};

    World<N> s;
    Ctx c = make_ctx(p, w, k == 0);
    World<N> v;
    if (active) {
        load_world(s, p, w);
        {
            Orig<N> o;
            capture(o, s);
            LaneOrig x;
            x.world = world_orig(o);
            x.agent = pick_by<N>(k, [&](int j) { return o.ag[j]; });
            park_words(tile, lane, x);
        }
    }
    // the policy's sampling uniforms for step k + 1 (they depend on the seed,
    // step, row and bucket only): drawn while the state loads are in flight,
    // off the bucket pass's chain
    BucketNoise<32> noise;
    if (!LAST && a.stochastic) bucket_noise<32>(noise, a.seed, a.step, w0, p.num_worlds, lane);
    // the workgroup's copy of the network (read after the barrier below)
    if (!LOOP) policy_weights_to_lds(S.wt, a.w, (int)threadIdx.x, WPG * WAVE);
    if (active) step_world_pre_obs(s, c, ag);
    if (active) {
        agent_view(s, v, k);
        sys_reward_agent(v, 0, AGENT0_ID + k);
        const LaneOrig x = unpark_words<LaneOrig>(tile, lane);
        store_world_agent<N, BB_COL_AUX>(v, p, w * N + k, 0, &x.agent);
        if (k == 0) {
            Orig<N> o;
            set_world_orig(o, x.world);
            store_world_shared<N, BB_COL_AUX>(s, p, w, &o);
        }
        if (k == trainee && a.reward) {  // buffer.rewards / not_dones source of step k
            a.reward[w] = v.rew[0];
            a.done[w] = v.done[0];
        }
    }
    const int32_t ib = active ? inbounder_id(s) : -1;
    const bool share = active && obs_sharable(s);
    SharedObs<N> sh;
    lane_shared_obs(v, c, active, sh);
    const bool fast = active && canonical_slots(v, 0);
    const uint64_t live = __ballot(active);
    char *obs = (char *)(p.c.obs + w0 * N * (int64_t)obs_width(N));                // wave-uniform
    char *rec = (!LAST && a.obs_rec) ? (char *)(a.obs_rec + w0 * (int64_t)POL_IN) : nullptr;
    const int pl = lane & 15, pq = lane >> 4;
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    wave_sync();  // the parked words are read
    ppo_emit_pass<0>(v, c, sh, active, fast, share, tile + lane * PPS_RS, ib);
    if (!LOOP) lds_barrier();  // the pass's rows, and the workgroup's weights, are in LDS
    else wave_sync();
    ppo_layer1_pass<0>(tile, S.wt, acc, trainee, pl, pq);
    ppo_flush_pass<0, LAST>(tile, obs, rec, live, trainee, lane);
    wave_sync();
    ppo_emit_pass<1>(v, c, sh, active, fast, share, tile + lane * PPS_RS, ib);
    wave_sync();
    ppo_layer1_pass<1>(tile, S.wt, acc, trainee, pl, pq);
    ppo_flush_pass<1, LAST>(tile, obs, rec, live, trainee, lane);
    wave_sync();
    if (LAST && !a.value) return;  // (wave-uniform; no barrier follows)
    // LayerNorm 1, layer 2, heads (the tile's first 32 x 33 floats), then the
    // bucket pass (its exchange right behind them)
    float (*lt)[33] = (float (*)[33])tile;
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
        ln_relu_to_tile(acc[mt][0], acc[mt][1], S.wt.cst[0][pl], S.wt.cst[0][pl + 16], S.wt.cst[1][pl],
                        S.wt.cst[1][pl + 16], S.wt.cst[2][pl], S.wt.cst[2][pl + 16], lt + 16 * mt, pl, pq);
    pol_wave_sync();
    policy_tail_lds2(S.wt, lt, pl, pq);
    if constexpr (LAST) {
        if (a.value && lane < 32 && w0 + lane < p.num_worlds) a.value[w0 + lane] = lt[lane][POL_LOGITS];
    } else {
        PolicyArgs pa{};
        pa.rows = p.num_worlds;
        pa.stochastic = a.stochastic;
        pa.seed = a.seed;
        pa.step = a.step;
        pa.actions = p.c.action + trainee * 6;
        pa.act_stride = N * 6;
        pa.act_out = a.act_out;
        pa.log_prob = a.log_prob;
        pa.value = a.value;
        BucketLds<32> &bl = *(BucketLds<32> *)(tile + 32 * 33);
        if (a.stochastic) bucket_pass_spread<32, true, 1>(pa, lt, w0, lane, bl, nullptr, &noise);
        else bucket_pass_spread<32, true, 0>(pa, lt, w0, lane, bl, nullptr, &noise);
    }
}

// The policy pass of step 0 inside k_rollout_ppo (what a k_policy launch on
// the trainee's sim rows did before it): the wave's 32 trainee rows from the
// sim's observation tensor into its tile in the two passes' layout (pass P:
// row floats i with ((i >> 4) & 1) == P and i < 104 at slot (i >> 5) * 16 +
// (i & 15), as PassSink leaves them), the same layer-1 chain steps, LayerNorms,
// layers and bucket pass as after every step (bit-identical to k_policy), the
// rows copied into buffer.obs[0].
template <int WPG>
__device__ __forceinline__ void ppo_pass0_wave(const Params &p, const PpoStepArgs &a, PpoStepLds<WPG> &S, int blk,
                                               int wave, int lane)
{
    constexpr int N = 2, OW = obs_width(N);
    static_assert(OW == POL_IN, "the 2-agent row is the policy's input");
    float *tile = S.tile[wave];
    const int64_t W = p.num_worlds;
    const int64_t w0 = ((int64_t)blk * WPG + wave) * (WAVE / N);
    const int trainee = a.trainee;
    const int pl = lane & 15, pq = lane >> 4;
    const float *src = p.c.obs + (w0 * N + trainee) * (int64_t)OW;  // row m at src + m * N * OW
    BucketNoise<32> noise;
    if (a.stochastic) bucket_noise<32>(noise, a.seed, a.step0, w0, W, lane);
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const auto pass = [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        constexpr int NPC = P == 0 ? 14 : 12;  // float4 pieces of the pass per row
        vf4 v[32 * NPC / WAVE];
        int slot[32 * NPC / WAVE];
#pragma unroll
        for (int it = 0; it < 32 * NPC / WAVE; it++) {
            const int f = it * WAVE + lane, m = f / NPC, t = f - m * NPC;
            const int i = 32 * (t >> 2) + 16 * P + 4 * (t & 3);  // the piece's first row float
            slot[it] = (2 * m + trainee) * PPS_RS + ((i >> 5) << 4) + (i & 15);
            v[it] = w0 + m < W ? *(const vf4 *)(src + (int64_t)m * N * OW + i) : vf4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int it = 0; it < 32 * NPC / WAVE; it++) *(vf4 *)(tile + slot[it]) = v[it];
        wave_sync();
        ppo_layer1_pass<P>(tile, S.wt, acc, trainee, pl, pq);
        wave_sync();
    };
    pass(std::integral_constant<int, 0>());
    pass(std::integral_constant<int, 1>());
    if (a.obs0) {  // buffer.obs[0]: the rows as read (the zero tail included)
#pragma unroll 4
        for (int it = 0; it < 32 * (OW / 4) / WAVE; it++) {
            const int f = it * WAVE + lane, m = f / (OW / 4), j = f - m * (OW / 4);
            if (w0 + m < W)
                *(vf4 *)(a.obs0 + (w0 + m) * (int64_t)OW + 4 * j) = *(const vf4 *)(src + (int64_t)m * N * OW + 4 * j);
        }
    }
    float (*lt)[33] = (float (*)[33])tile;
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
        ln_relu_to_tile(acc[mt][0], acc[mt][1], S.wt.cst[0][pl], S.wt.cst[0][pl + 16], S.wt.cst[1][pl],
                        S.wt.cst[1][pl + 16], S.wt.cst[2][pl], S.wt.cst[2][pl + 16], lt + 16 * mt, pl, pq);
    pol_wave_sync();
    policy_tail_lds2(S.wt, lt, pl, pq);
    PolicyArgs pa{};
    pa.rows = W;
    pa.stochastic = a.stochastic;
    pa.seed = a.seed;
    pa.step = a.step0;
    pa.actions = p.c.action + trainee * 6;
    pa.act_stride = N * 6;
    pa.act_out = a.act0;
    pa.log_prob = a.log_prob0;
    pa.value = a.value0;
    BucketLds<32> &bl = *(BucketLds<32> *)(tile + 32 * 33);
    if (a.stochastic) bucket_pass_spread<32, true, 1>(pa, lt, w0, lane, bl, nullptr, &noise);
    else bucket_pass_spread<32, true, 0>(pa, lt, w0, lane, bl, nullptr, &noise);
    wave_sync();  // the tile is rewritten by step 0
}

template <int WPG, bool LAST>
__global__ __launch_bounds__(WAVE * WPG, 2) void k_step_ppo(const Params p, const PpoStepArgs a)
{
    if constexpr (BB_N == 2) {
        __shared__ PpoStepLds<WPG> S;
        const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE);
        ppo_step_wave<WPG, LAST>(p, a, S, (int)blockIdx.x, wave, (int)threadIdx.x % WAVE);
    }
}

// k_rollout_ppo<2>: the steps of k_step_ppo for a whole rollout in one launch.
// Worlds are independent, so each wave runs its 32 worlds' K steps back to
// back -- the state stored at the end of a step and loaded at the start of
// the next, the trainee's actions through the sim's action column, as between
// k_step_ppo launches -- with no kernel boundary between steps and no
// barrier: waves drift apart, and the policy's MFMA phase of one overlaps
// another's systems.  A wave reads only what its own lanes wrote (same wave,
// same vector L1: coherent; the fence orders the store and the loads).  Each
// step computes exactly what k_step_ppo computes (bit-identical).
template <int WPG>
__global__ __launch_bounds__(WAVE * WPG, 2) void k_rollout_ppo(const Params p, const PpoStepArgs a0, int32_t steps)
{
    if constexpr (BB_N == 2) {
        __shared__ PpoStepLds<WPG> S;
        const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE);
        const int lane = (int)threadIdx.x % WAVE;
        policy_weights_to_lds(S.wt, a0.w, (int)threadIdx.x, WPG * WAVE);
        lds_barrier();
        if (a0.pass0) {
            ppo_pass0_wave<WPG>(p, a0, S, (int)blockIdx.x, wave, lane);
            // step 0 reads the action column the pass wrote
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
        const int64_t W = p.num_worlds;
        for (int32_t k = 0; k < steps; k++) {
            // opaque per-step copies of the indices: nothing derived from them
            // (column addresses, the world's keys) is computed before the loop
            // and held across it
            int32_t k_t = k, blk_t = (int)blockIdx.x, wave_t = wave, lane_t = lane;
            __asm__ volatile("" : "+s"(k_t), "+s"(blk_t), "+s"(wave_t));
            __asm__ volatile("" : "+v"(lane_t));
            const PpoStepArgs a = ppo_loop_args(a0, k_t, steps, W);
            if (k_t + 1 < steps) ppo_step_wave<WPG, false, true>(p, a, S, blk_t, wave_t, lane_t);
            else ppo_step_wave<WPG, true, true>(p, a, S, blk_t, wave_t, lane_t);
            // this step's state / action stores before the next step's loads
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
    }
}

// ------------------------------------------------------------------ N >= 4
// One lane per agent; the world's state lives in LDS and its N lanes run the
// world-level systems on it together (same instructions, same values); the
// per-agent systems are computed by the agent's lane and exchanged through
// an LDS buffer (LdsAgents).  No per-lane copy of the world: nothing to spill.
#ifndef BB_OBS_PIECES
#define BB_OBS_PIECES 1
#endif
#ifndef BB_SHARED_TILE
#define BB_SHARED_TILE 0
#endif
#ifndef BB_XW
#define BB_XW ((BB_OBS_PIECES && !BB_SHARED_TILE) ? 13 : 33)
#endif
// Words per lane in the exchange buffer (>= the systems' per-agent results;
// >= Intrinsic where the observation pass exchanges intrinsic blocks through
// it).  Odd, so that the rows lanes of different worlds read at once fall in
// different LDS banks
// (at 32 words the row start is 0 or 32 mod 64 banks: up to 30-way conflicts).
constexpr int XW = BB_XW;

template <int N, int MODE>
struct LdsAgents {
    int k, slot;
    uint32_t (*x)[XW];
    const Params *p;
    template <class T, int NN, class F>
    __device__ void all(F f, T (&out)[NN]) const
    {
        static_assert(NN == N && sizeof(T) <= XW * 4, "exchange slot");
        const T mine = f(k);
        __syncthreads();  // earlier readers of the buffer are done
        __builtin_memcpy(x[slot * N + k], &mine, sizeof(T));
        __syncthreads();
#pragma unroll
        for (int j = 0; j < N; j++) __builtin_memcpy(&out[j], x[slot * N + j], sizeof(T));
    }
    // The world is in LDS: each lane applies its own agent's result (no
    // exchange; agent i's f reads nothing another agent's apply writes, and
    // the wave's reads all precede its writes in program order).  Lanes past
    // the last world mirror its agents and write the same values.
    template <int NN, class F, class P>
    __device__ void each(F f, P apply) const
    {
        static_assert(NN == N, "one lane per agent");
        apply(k, f(k));
        __syncthreads();
    }
    __device__ void mark(int point) const { trace_point<MODE>(*p, point); }
};

// ---- observation rows as whole-wave pieces (N >= 4) -------------------------
// A wave's WPW worlds own WPW*N consecutive observation rows.  After the
// systems, each world's lanes write the row *sources* into an LDS table
// (ObsSrc, overlaying the then dead world state and exchange buffer): the two
// team contexts (obs 0-22), every agent's position and intrinsic block, the
// observer-to-agent direction/distance matrix and the one-hot tails.  A
// per-float decode table (PieceCode, row position i -> table entry as a
// function of the observer a) lets the wave write its rows as consecutive
// 16-byte pieces -- 1 KB of whole lines per store instruction instead of one
// 16-byte piece of each of 64 rows -- every float bit-identical to
// emit_row_view.  Only worlds whose rows share the intrinsic blocks
// (obs_sharable: every generated world) take this path.
template <int N>
struct ObsSrc {
    static constexpr int QR = obs_width(N) / 4;   // 16-byte pieces per row
    static constexpr int CTX = 0;                 // [2][23] context of a team-0 / team-1 observer
    static constexpr int PI = 46;                 // [N][34] position (3) + intrinsic block (31)
    static constexpr int R = PI + 34 * N;         // [N][N-1][4] direction (3) + distance a -> j, j != a
    static constexpr int OH = R + 4 * N * (N - 1);  // [2N] holder one-hot, inbounder one-hot
    static constexpr int TM = OH + 2 * N;         // [N] team(a) != 0 (int bits)
    static constexpr int Z = TM + N;              // one zero
    static constexpr int ES = (Z + 4) & ~3;       // floats per world (whole 4-entry groups: esw stays inside)
};

// code[i] for row float i: entry = base + MA*a + MJ*(T ? t : j) + MT*team(a),
// with j = t + (t >= a) the agent in other-agent block t of observer a:
// bits 0-9 base, 10-15 MA, 16-21 MJ, 22-26 MT, 27 T, 28-31 t.
template <int N>
struct PieceCode {
    uint32_t c[obs_width(N)];
};
template <int N>
constexpr uint32_t piece_code(int i)
{
    using S = ObsSrc<N>;
    static_assert(S::Z < 1024 && 4 * (N - 1) < 64 && N <= 16, "code fields");
    const int tail = 61 + 38 * (N - 1);
    auto code = [](int base, int ma, int mj, int mt, int t, int tsel = 0) {
        return (uint32_t)base | ((uint32_t)ma << 10) | ((uint32_t)mj << 16) | ((uint32_t)mt << 22)
               | ((uint32_t)tsel << 27) | ((uint32_t)t << 28);
    };
    if (i < 23) return code(S::CTX + i, 0, 0, 23, 0);
    if (i < 26) return code(S::PI + (i - 23), 34, 0, 0, 0);
    if (i < 30) return code(S::Z, 0, 0, 0, 0);
    if (i < 61) return code(S::PI + 3 + (i - 30), 34, 0, 0, 0);
    if (i < tail) {
        const int u = i - 61, t = u / 38, f = u % 38;
        if (f < 3) return code(S::PI + f, 0, 34, 0, t);
        if (f < 7) return code(S::R + (f - 3), 4 * (N - 1), 4, 0, t, 1);  // row a, column t
        return code(S::PI + 3 + (f - 7), 0, 34, 0, t);
    }
    if (i < tail + 2 * N) return code(S::OH + (i - tail), 0, 0, 0, 0);
    return code(S::Z, 0, 0, 0, 0);
}
template <int N>
constexpr PieceCode<N> make_piece_code()
{
    PieceCode<N> m{};
    for (int i = 0; i < obs_width(N); i++) m.c[i] = piece_code<N>(i);
    return m;
}
template <int N>
__constant__ PieceCode<N> PIECE_CODE = make_piece_code<N>();

// Table entries are stored swizzled: bits 0-1 of the index XOR bits 5-6, so
// that the 4-float stride of consecutive lanes' pieces (lane L reads entry
// ~4L + c) spreads over all 32 banks instead of 8 (4-way conflicts).
__device__ __forceinline__ int esw(int i) { return i ^ ((i >> 5) & 3); }

template <int N>
__device__ __forceinline__ int piece_src(uint32_t code, int a, int tm)
{
    const int t = (int)(code >> 28);
    const int j = ((code >> 27) & 1u) ? t : t + (t >= a ? 1 : 0);
    return (int)(code & 0x3FFu) + (int)((code >> 10) & 0x3Fu) * a + (int)((code >> 16) & 0x3Fu) * j
           + (int)((code >> 22) & 0x1Fu) * tm;
}

// N = 4: a world's agents are the 4 lanes of a DPP quad, so the per-agent
// results are exchanged by quad_perm moves (LaneAgents) instead of through an
// LDS buffer: 3.3 KB less LDS per wave, 12 waves per CU instead of 9.
#ifndef BB_DPP_AGENTS
#define BB_DPP_AGENTS 1
#endif
template <int N>
struct DppAgents {
    static constexpr bool value = BB_DPP_AGENTS && N == 4 && XW < INTRINSIC;
};

// The observation pass writes the row-source table for OBS_PARTS groups of
// the wave's worlds in turn (a group's rows emitted before the next group's
// sources overlay them), so the table needs room for WPW / OBS_PARTS worlds
// only: at N = 4 it was the largest part of a wave's LDS (15.6 of 16.4 KB:
// 10 waves per CU; with 2 parts 13.5 KB: 12, the VGPR bound).
#ifndef BB_OBS_PARTS
#define BB_OBS_PARTS 1
#endif
template <int N>
struct SharedLds {
    static constexpr int WPW = WAVE / N;  // worlds per wave
    // (N = 4 only: the lanes of a later part keep their sources in registers
    // meanwhile -- at N = 10 that is 160 -> 256 VGPRs, no occupancy gained)
    static constexpr int PARTS = N == 4 ? (BB_OBS_PARTS < WPW ? BB_OBS_PARTS : WPW) : 1;
    static constexpr int SPP = (WPW + PARTS - 1) / PARTS;  // world slots per source-table part
    union {
        struct {
            World<N> world[WPW];
            uint32_t x[DppAgents<N>::value ? 1 : WAVE][XW];  // systems: per-agent exchange
        };
        float e[SPP][ObsSrc<N>::ES];           // observation pass: row sources of one part
    };
    uint4 code[BB_OBS_PIECES ? obs_width(N) / 4 : 1];  // PieceCode, 4 codes per piece
};

// The lane's sources (agent k of its world), computed from the world state
// into registers; written into the table by put() once every lane is done
// reading the state the table overlays.  Position and intrinsic block
// always (the direct row of a non-sharable world reads them too).
template <int N>
struct LaneSources {
    float pi[34];
    float r[N][4];
    float ctx[23];
    float oh_holder, oh_inb;
    int32_t tm;
    bool first;  // lowest agent of its team: writes the team's context

    __device__ __forceinline__ void compute(const World<N> &s, const Ctx &c, int k, int32_t ib, bool share)
    {
        {
            ArraySink<34> o;
            o.idx = 0;
            o.put3(s.pos(k));
            emit_intrinsic(s, o, k, attacking_hoop(s, c, k));
#pragma unroll
            for (int q = 0; q < 34; q++) pi[q] = o.v[q];
        }
        if (!share) return;
        const F3 p = s.pos(k);
#pragma unroll
        for (int j = 0; j < N; j++) {
            const F3 to = s.pos(j) - p;  // as emit_row_view
            const float l2 = len2(to);
            const float rr = 1.0f / bbm::sqrtf_(l2);
            const F3 d = l2 > 1e-6f ? to * rr : f3(0.f, 0.f, 0.f);
            r[j][0] = d.x; r[j][1] = d.y; r[j][2] = d.z; r[j][3] = bbm::sqrtf_(l2);
        }
        oh_holder = AGENT0_ID + k == s.holder ? 1.f : 0.f;
        oh_inb = AGENT0_ID + k == ib ? 1.f : 0.f;
        tm = s.team[k] != 0 ? 1 : 0;
        first = true;
#pragma unroll
        for (int j = 0; j < N; j++) first &= !(j < k && s.team[j] == s.team[k]);
        if (first) {
            ArraySink<23> o;
            o.idx = 0;
            F3 att, dfn;
            obs_context(s, c, o, k, &att, &dfn);
#pragma unroll
            for (int q = 0; q < 23; q++) ctx[q] = o.v[q];
        }
    }

    __device__ __forceinline__ void put(float *e, int k, bool share) const
    {
        using S = ObsSrc<N>;
#pragma unroll
        for (int q = 0; q < 34; q++) e[esw(S::PI + 34 * k + q)] = pi[q];
        if (!share) return;
#pragma unroll
        for (int j = 0; j < N; j++)
            if (j != k)
#pragma unroll
                for (int q = 0; q < 4; q++) e[esw(S::R + 4 * (k * (N - 1) + (j > k ? j - 1 : j)) + q)] = r[j][q];
        e[esw(S::OH + k)] = oh_holder;
        e[esw(S::OH + N + k)] = oh_inb;
        e[esw(S::TM + k)] = bitsf((uint32_t)tm);
        if (first)
#pragma unroll
            for (int q = 0; q < 23; q++) e[esw(S::CTX + 23 * tm + q)] = ctx[q];
        if (k == 0) e[esw(S::Z)] = 0.f;
    }
};

// The wave's rows [row0, row0 + WPW*N) whose bit is set in `rows`: lane L
// writes pieces L, L + 64, ... of each row (the row's bytes in 1 KB of
// consecutive pieces per store instruction).  A lane's pieces sit at the same
// row positions in every row, so their table entries are decoded once, per
// observer a, before the loop: per piece 4 LDS reads and one store.  The
// row's team (obs 0-22 entries) is bit r of `teams` (a ballot taken when the
// sources were computed): a wave-uniform offset with no LDS read.
// Rows go in read batches of RB rows; the reads of the next batch are issued
// before this batch's stores (only the stores are predicated on the row's
// bit), so the LDS latency hides under the stores -- row by row, each row's
// store waited on its own reads (and on a read of its team before them).
// Slots [S0, S1) of the wave's worlds, whose sources are at sm.e[slot - S0].
#ifndef BB_OBS_RB
#define BB_OBS_RB 0  // rows per read batch (0: a slot's N rows at one piece per row, else 2)
#endif
template <int N, int NP, int RB, int A0>
__device__ __forceinline__ void read_batch(const float *e, const int (&src)[NP][N][4], const int (&dtm)[NP][4],
                                           uint64_t tbits, vf4 (&v)[RB][NP])
{
#pragma unroll
    for (int b = 0; b < RB; b++) {
        const int tm = -(int)((tbits >> (A0 + b)) & 1ull);  // team 1: all ones
#pragma unroll
        for (int p = 0; p < NP; p++)
            v[b][p] = vf4{e[src[p][A0 + b][0] + (dtm[p][0] & tm)], e[src[p][A0 + b][1] + (dtm[p][1] & tm)],
                          e[src[p][A0 + b][2] + (dtm[p][2] & tm)], e[src[p][A0 + b][3] + (dtm[p][3] & tm)]};
    }
}
template <int N, int AUX, int S0, int S1, int NP, int RB, int A0, class SM>
__device__ __forceinline__ void emit_slot_batches(const SM &sm, const int (&src)[NP][N][4],
                                                  const int (&dtm)[NP][4], uint64_t rows, uint64_t teams, char *base,
                                                  int lane, int slot, vf4 (&cur)[RB][NP])
{
    constexpr int QR = ObsSrc<N>::QR;
    vf4 nxt[RB][NP];
    if constexpr (A0 + RB < N) {
        read_batch<N, NP, RB, A0 + RB>(sm.e[slot - S0], src, dtm, teams >> (slot * N), nxt);
    } else {
        if (slot + 1 < S1) read_batch<N, NP, RB, 0>(sm.e[slot + 1 - S0], src, dtm, teams >> ((slot + 1) * N), nxt);
    }
#pragma unroll
    for (int b = 0; b < RB; b++) {
        const int r = slot * N + A0 + b;
        if (!((rows >> r) & 1ull)) continue;  // wave-uniform
#pragma unroll
        for (int p = 0; p < NP; p++)
            if (p * WAVE + lane < QR) row_store<AUX>(base, ((uint32_t)r * QR + p * WAVE + lane) * 16u, cur[b][p]);
    }
#pragma unroll
    for (int b = 0; b < RB; b++)
#pragma unroll
        for (int p = 0; p < NP; p++) cur[b][p] = nxt[b][p];
    if constexpr (A0 + RB < N)
        emit_slot_batches<N, AUX, S0, S1, NP, RB, A0 + RB, SM>(sm, src, dtm, rows, teams, base, lane, slot, cur);
}
template <int N, int AUX, int S0, int S1, class SM>
__device__ __forceinline__ void emit_pieces_rows(const SM &sm, uint64_t rows, uint64_t teams, float *obs,
                                                 int64_t row0, int lane)
{
    using S = ObsSrc<N>;
    constexpr int WPW = SM::WPW, QR = S::QR, NP = (QR + WAVE - 1) / WAVE;
    constexpr int RB = (BB_OBS_RB > 0 && N % (BB_OBS_RB > 0 ? BB_OBS_RB : 1) == 0) ? BB_OBS_RB : (NP == 1 ? N : 2);
    static_assert(N % RB == 0, "whole read batches per slot");
    int src[NP][N][4], dtm[NP][4];
#pragma unroll
    for (int p = 0; p < NP; p++) {
        const int q = p * WAVE + lane;
        const uint4 cd = sm.code[q < QR ? q : 0];
        const uint32_t code[4] = {cd.x, cd.y, cd.z, cd.w};
#pragma unroll
        for (int c = 0; c < 4; c++) {
#pragma unroll
            for (int a = 0; a < N; a++) src[p][a][c] = esw(piece_src<N>(code[c], a, 0));
            dtm[p][c] = esw(piece_src<N>(code[c], 0, 1)) - esw(piece_src<N>(code[c], 0, 0));  // context entries only
        }
    }
    char *base = (char *)(obs + row0 * obs_width(N));  // wave-uniform
    static_assert(S1 <= WPW && S1 - S0 <= SM::SPP, "part of the source table");
    vf4 cur[RB][NP];
    read_batch<N, NP, RB, 0>(sm.e[0], src, dtm, teams >> (S0 * N), cur);
    for (int slot = S0; slot < S1; slot++)
        emit_slot_batches<N, AUX, S0, S1, NP, RB, 0, SM>(sm, src, dtm, rows, teams, base, lane, slot, cur);
}

template <int N, int AUX, int S0, int S1, class SM>
__device__ __forceinline__ void emit_pieces(const SM &sm, uint64_t rows, uint64_t teams, float *obs,
                                            int64_t row0, int lane)
{
    emit_pieces_rows<N, AUX, S0, S1, SM>(sm, rows, teams, obs, row0, lane);
}

// The source table written and emitted part by part (BB_OBS_PARTS): the
// world state is dead once every lane holds its sources; each part's lanes
// put theirs, the wave emits that part's rows, and the next part overlays it.
template <int N, int AUX, int P = 0, class SM = SharedLds<N>>
__device__ __forceinline__ void obs_parts(SM &sm, const LaneSources<N> &src, uint64_t rows, uint64_t teams, float *obs,
                                          int64_t row0, int lane, int slot, int k, bool active, bool share)
{
    using SL = SM;
    constexpr int S0 = P * SL::SPP, S1 = (S0 + SL::SPP < SL::WPW) ? S0 + SL::SPP : SL::WPW;
    __syncthreads();  // the world state (or the previous part) is dead: this part overlays it
    if (active && slot >= S0 && slot < S1) src.put(sm.e[slot - S0], k, share);
    __syncthreads();
    emit_pieces<N, AUX, S0, S1, SM>(sm, rows, teams, obs, row0, lane);
    if constexpr (P + 1 < SL::PARTS) obs_parts<N, AUX, P + 1, SM>(sm, src, rows, teams, obs, row0, lane, slot, k, active, share);
}

template <int N, int MODE, int PHASE = 0>
__device__ __forceinline__ void obs_phases_view(const World<N> &s, const Ctx &c, int k, const uint32_t (*x)[XW],
                                                int slot, bool share, bool fast, float *tile, int64_t row0,
                                                int lane, int32_t ib)
{
    using T = PhasedTile<N>;
    if (fast) {
        constexpr int LO = PHASE * T::QP * 4, HI = LO + T::QP * 4;
        WindowSink<LO, HI> o;
        o.row = tile + lane * T::RS; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
        auto intr = [&](int j, int q) { return bitsf(x[slot * N + j][q]); };
        emit_row_view(s, c, k, intr, share, o, ib);
    }
    __syncthreads();
    constexpr int Q0 = PHASE * T::QP, QN = (T::QW - Q0 < T::QP) ? T::QW - Q0 : T::QP;
    constexpr int QZ = T::QU - Q0 < 0 ? 0 : (T::QU - Q0 < QN ? T::QU - Q0 : QN);
    flush_tile<N, T::QP, T::RS, Q0, QN, 1, QZ>(tile, c.p->c.obs, row0, __ballot(fast), lane);
    if constexpr (PHASE + 1 < T::PH) {
        __syncthreads();
        obs_phases_view<N, MODE, PHASE + 1>(s, c, k, x, slot, share, fast, tile, row0, lane, ib);
    }
}

template <int N>
struct SharedTiled {
    static constexpr bool value = BB_SHARED_TILE != 0;
};

// BEYOND: the step's bytes far exceed the Infinity Cache -- rows and columns
// are stored non-temporally (see BB_SHARED_BEYOND_AUX).
template <int N, int MODE, bool BEYOND = false>
__device__ __forceinline__ void step_shared_world(const Params &p, float *tile, SharedLds<N> &sm, int blk, int lane)
{
    constexpr int AUX = BEYOND ? BB_SHARED_BEYOND_AUX : BB_SHARED_AUX;
    constexpr int CAUX = BEYOND ? BB_SHARED_BEYOND_COL_AUX : BB_SHARED_AUX;
    constexpr int WPW = SharedLds<N>::WPW, OW = obs_width(N);
    // lanes past WPW*N mirror agents of the last world: they run its systems
    // (identical LDS writes) but own no row and store nothing
    const bool lane_used = lane < WPW * N;
    const int slot = lane_used ? lane / N : WPW - 1;
    const int k = lane_used ? lane % N : (lane - WPW * N) % N;
    const int64_t w0 = (int64_t)blk * WPW;
    const int64_t w = w0 + slot;
    const bool world_ok = w < p.num_worlds;  // uniform over the world's lanes
    const bool active = lane_used && world_ok;
    World<N> &s = sm.world[slot];
    using AG = typename std::conditional<DppAgents<N>::value, LaneAgents<N, MODE, true>, LdsAgents<N, MODE>>::type;
    AG ag;
    if constexpr (DppAgents<N>::value) ag = LaneAgents<N, MODE, true>{k, &p};
    else ag = LdsAgents<N, MODE>{k, slot, sm.x, &p};
    Ctx c = make_ctx(p, w, active && k == 0);
    trace_point<MODE>(p, 0);
    constexpr bool PIECES = BB_OBS_PIECES && MODE != MODE_DIRECT_OBS && !SharedTiled<N>::value;

    if constexpr (BB_PRIO_LOAD > 0) __builtin_amdgcn_s_setprio(BB_PRIO_LOAD);
    if (active) {
        // every load issued before the first LDS write (one memory latency)
        AgentRaw<N> ar;
        WorldRaw wr;
        ar.load(p, w, k);
        if (k == 0) wr.load(p, w);
        ar.commit(s, k);
        if (k == 0) wr.commit(s);
    }
    __syncthreads();
    if constexpr (BB_PRIO_LOAD > 0) __builtin_amdgcn_s_setprio(0);
    // event-only words as loaded (store only on change, see Orig)
    LaneOrig lo;
    if (active) {
        Orig<N> o;
        game_words(s, o.game);
        phys_words(s, o.phys);
        o.grab[0] = (uint32_t)s.grab; o.grab[1] = (uint32_t)s.holder;
        o.clock = (uint32_t)s.reset_now; o.rng = s.rng_ctr;
        lo.world = world_orig(o);
        lo.agent = orig_agent(s, k);
    }
    if constexpr (MODE == MODE_SKIP) step_world_pre_obs(s, c, ag, p.diag_skip, 0u);
    else if constexpr (MODE != MODE_IO && MODE != MODE_IO_OBS) step_world_pre_obs(s, c, ag);
    __syncthreads();
    trace_point<MODE>(p, 7);
    trace_resets<MODE>(p, active, s);
    // reward (own agent) and state columns
    if constexpr (MODE != MODE_IO && MODE != MODE_IO_OBS) {
        const float r = reward_one(s, k, AGENT0_ID + k);
        __syncthreads();  // every lane has read the rewards it needs
        if (lane_used) s.rew[k] = r;
        __syncthreads();
    }
    if (active) {
        store_world_agent<N, CAUX>(s, p, w * N + k, k, &lo.agent);
        if (k == 0) {
            Orig<N> o;
            set_world_orig(o, lo.world);
            store_world_shared<N, CAUX>(s, p, w, &o);
        }
    }
    trace_point<MODE>(p, 8);
    if constexpr (MODE == MODE_IO || MODE == MODE_NO_OBS) return;

    const int32_t ib = inbounder_id(s);
    const bool share = obs_sharable(s);
    if constexpr (PIECES) {
        LaneSources<N> src;
        if (active) {
            src.compute(s, c, k, ib, share);
            if (!share) {  // rows the pieces do not cover: straight from the lane
                float *grow = p.c.obs + (w * N + k) * (int64_t)OW;
                if (canonical_slots(s, k)) {
                    fill_obs_fast(s, c, k, grow, ib);
                } else {
                    fill_obs_slow(s, c, k, grow, ib);
                }
            }
        }
        const uint64_t rows = __ballot(active && share);
        const uint64_t teams = __ballot(active && share && src.tm != 0);  // bit r: row r's observer in team 1
        // the row pass (memory-bound) ahead of other waves' systems (VALU)
        if constexpr (BB_PRIO_ROWS > 0) __builtin_amdgcn_s_setprio(BB_PRIO_ROWS);
        obs_parts<N, AUX>(sm, src, rows, teams, p.c.obs, w0 * N, lane, slot, k, active, share);
        trace_point<MODE>(p, 9);
        return;
    }
    if constexpr (XW < INTRINSIC) {
        // (diagnostic modes of a piece build) no room in the exchange buffer
        // for intrinsic blocks: each lane writes its row alone
        if (active) {
            float *grow = p.c.obs + (w * N + k) * (int64_t)OW;
            if (canonical_slots(s, k)) fill_obs_fast(s, c, k, grow, ib);
            else fill_obs_slow(s, c, k, grow, ib);
        }
        trace_point<MODE>(p, 9);
        return;
    } else {
    // observations: intrinsic block of the lane's agent into the exchange
    // buffer, then the row in passes through the tile
    {
        ArraySink<INTRINSIC> o;
        o.idx = 0;
        emit_intrinsic(s, o, k, attacking_hoop(s, c, k));
        __syncthreads();  // exchange-buffer readers are done
        if (lane_used) {
#pragma unroll
            for (int q = 0; q < INTRINSIC; q++) sm.x[lane][q] = fbits(o.v[q]);
        }
        __syncthreads();
    }
    const bool fast = active && canonical_slots(s, k);
    // rows straight from the lanes (no tile: the LDS goes to occupancy) unless
    // BB_SHARED_TILE stages them
    if constexpr (MODE == MODE_DIRECT_OBS || !SharedTiled<N>::value) {
        if (active) {
            float *grow = p.c.obs + (w * N + k) * (int64_t)OW;
            if (fast) {
                RowSink o;
                o.row = grow; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
                auto intr = [&](int j, int q) { return bitsf(sm.x[slot * N + j][q]); };
                emit_row_view(s, c, k, intr, share, o, ib);
            } else {
                fill_obs_slow(s, c, k, grow, ib);
            }
        }
    } else {
        if (active && !fast) fill_obs_slow(s, c, k, p.c.obs + (w * N + k) * (int64_t)OW, ib);
        obs_phases_view<N, MODE>(s, c, k, sm.x, slot, share, fast, tile, w0 * N, lane, ib);
    }
    trace_point<MODE>(p, 9);
    }
}

// K steps per launch with the world in LDS (bb_rollout at N >= 4, SURVEY
// 8(f) rank 4; scripts/ppo.py:65): step_shared_world's step K times over the
// world the wave loaded once.  Per step only the action rows come in
// (actions[t], the defence AI's overrides written back there, as the per-step
// launches leave them) and the observation rows, rewards and done flags go
// out (obs/reward/done + t * step); the state columns are stored once, after
// the last step.  The row-source table of the observation pass overlays the
// world state (SharedLds), so each lane keeps 1/N of the world's words in
// registers across the pass and writes them back after it.
// At N >= 6 the register copy (45+ words per lane on top of the row pass's
// row sources and decode tables) spills: there the source table sits beside
// the world instead (SharedLdsRoll: more LDS per wave, fewer waves per CU).
template <int N>
struct SharedLdsRoll {
    static constexpr int WPW = WAVE / N, PARTS = 1, SPP = WPW;
    World<N> world[WPW];
    uint32_t x[DppAgents<N>::value ? 1 : WAVE][XW];
    float e[SPP][ObsSrc<N>::ES];
    uint4 code[obs_width(N) / 4];
};
template <int N>
struct SharedRollout {
    static constexpr bool value = Lanes<N>::SHARED && BB_OBS_PIECES && !SharedTiled<N>::value;
    static constexpr bool KEEP = N == 4;  // the world's words in registers across the row pass (else SharedLdsRoll)
    static constexpr int WORDS = (int)(sizeof(World<N>) / 4);
    static constexpr int CH = KEEP ? (WORDS + N - 1) / N : 1;  // words a lane keeps across the row pass
    using Lds = typename std::conditional<KEEP, SharedLds<N>, SharedLdsRoll<N>>::type;
};

// STORE: bb_step_n_staged's resident loop (RolloutArgs::store_state) -- every
// step stores the state columns with k_step_shared's cache policies (taken
// only while the step's bytes fit the Infinity Cache, bb::resident_staged),
// rows into the sim's tensor.
template <int N, class SM, bool STORE = false>
__device__ __forceinline__ void rollout_shared_world(const Params &p, const RolloutArgs &r, SM &sm)
{
    using SR = SharedRollout<N>;
    constexpr int WPW = SM::WPW, OW = obs_width(N);
    // rows into a fresh [K][W][N][OBSW] buffer, or (STORE) as the step's
    constexpr int AUX = !STORE ? BB_ROLLOUT_AUX : BB_SHARED_AUX;
    constexpr int CAUX = BB_SHARED_AUX;
    const int lane = threadIdx.x;
    const bool lane_used = lane < WPW * N;
    const int slot = lane_used ? lane / N : WPW - 1;
    const int k = lane_used ? lane % N : (lane - WPW * N) % N;
    const int64_t w0 = (int64_t)blockIdx.x * WPW;
    const int64_t w = w0 + slot;
    const int64_t W = p.num_worlds;
    const bool world_ok = w < W;
    const bool active = lane_used && world_ok;
    World<N> &s = sm.world[slot];
    using AG = typename std::conditional<DppAgents<N>::value, LaneAgents<N, MODE_FULL, true>, LdsAgents<N, MODE_FULL>>::type;
    AG ag;
    if constexpr (DppAgents<N>::value) ag = LaneAgents<N, MODE_FULL, true>{k, &p};
    else ag = LdsAgents<N, MODE_FULL>{k, slot, sm.x, &p};
    if (active) {
        AgentRaw<N> ar;
        WorldRaw wr;
        ar.load(p, w, k);
        if (k == 0) wr.load(p, w);
        ar.commit(s, k);
        if (k == 0) wr.commit(s);
    }
    for (int t = 0; t < r.steps; t++) {
        // per-step opaque copies of the lane's indices: what derives from them
        // (the row pass's decode tables, column addresses) is recomputed in
        // the iteration instead of being hoisted out of the loop and held in
        // registers across every step (k_rollout's discipline)
        int lane_t = lane, k_t = k;
        int64_t w_t = w;
        __asm__ volatile("" : "+v"(lane_t));
        __asm__ volatile("" : "+v"(k_t));
        __asm__ volatile("" : "+v"(w_t));
        const int64_t row = w_t * N + k_t;  // the lane's agent row
        Ctx c = make_ctx(p, w_t, active && k_t == 0);
        // the action row of step t (actions[t] stands in for the action column)
        int32_t *acts = r.actions + (int64_t)t * W * N * 6;
        if (active) {
            uint32_t a6[6];
            load_words<6>(acts, row, a6);
#pragma unroll
            for (int q = 0; q < 6; q++) s.act[k_t][q] = (int32_t)a6[q];
        }
        __syncthreads();
        step_world_pre_obs(s, c, ag);
        __syncthreads();
        const float rw = reward_one(s, k_t, AGENT0_ID + k_t);
        __syncthreads();  // every lane has read the rewards it needs
        if (lane_used) s.rew[k_t] = rw;
        __syncthreads();
        if (active) {
            if constexpr (STORE) {
                // every column of step t as k_step stores it: the action row
                // (overrides included) into actions[t], reward / done into the
                // sim's columns (r.reward / r.done here)
                Params ps = p;
                ps.c.action = acts;
                store_world_agent<N, CAUX>(s, ps, row, k_t);
                if (k_t == 0) store_world_shared<N, CAUX>(s, p, w_t);
            } else {
                uint32_t a6[6];
#pragma unroll
                for (int q = 0; q < 6; q++) a6[q] = (uint32_t)s.act[k_t][q];
                store_words<6>(acts, row, a6);  // with the defence AI's overrides
                r.reward[(int64_t)t * r.rd_step + row] = s.rew[k_t];
                r.done[(int64_t)t * r.rd_step + row] = s.done[k_t];
            }
        }
        // observation rows of step t
        float *obs_t = r.obs + (int64_t)t * r.obs_step;
        const int32_t ib = inbounder_id(s);
        const bool share = obs_sharable(s);
        LaneSources<N> src;
        if (active) {
            src.compute(s, c, k_t, ib, share);
            if (!share) {  // rows the pieces do not cover: straight from the lane
                float *grow = obs_t + row * (int64_t)OW;
                if (canonical_slots(s, k_t)) fill_obs_fast(s, c, k_t, grow, ib);
                else fill_obs_slow(s, c, k_t, grow, ib);
            }
        }
        const uint64_t rows = __ballot(active && share);
        const uint64_t teams = __ballot(active && share && src.tm != 0);
        // the lane's share of the world's words, kept across the row pass
        // (whose source table overlays the world)
        uint32_t keep[SR::CH];
        if constexpr (SR::KEEP) {
            const uint32_t *ws = (const uint32_t *)&s;
#pragma unroll
            for (int i = 0; i < SR::CH; i++) {
                const int idx = k_t * SR::CH + i;
                keep[i] = idx < SR::WORDS ? ws[idx] : 0u;
            }
        }
        obs_parts<N, AUX, 0, SM>(sm, src, rows, teams, obs_t, w0 * N, lane_t, slot, k_t, active, share);
        __syncthreads();  // the table's readers are done
        if constexpr (SR::KEEP) {
            if (lane_used) {
                uint32_t *ws = (uint32_t *)&s;
#pragma unroll
                for (int i = 0; i < SR::CH; i++) {
                    const int idx = k_t * SR::CH + i;
                    if (idx < SR::WORDS) ws[idx] = keep[i];
                }
            }
            __syncthreads();
        }
    }
    if (STORE && active && r.steps > 0) {  // the last step's action rows into the sim's action tensor
        int k_e = k;
        int64_t w_e = w;
        __asm__ volatile("" : "+v"(k_e));
        __asm__ volatile("" : "+v"(w_e));
        uint32_t a6[6];
        load_words<6>(r.actions + (int64_t)(r.steps - 1) * p.num_worlds * N * 6, w_e * N + k_e, a6);
        store_words<6>(p.c.action, w_e * N + k_e, a6);
    }
    // the state after the last step, every column (the per-step launches'
    // last stores; actions / rewards / done flags as the last step left them)
    if (!STORE && active) {
        // (opaque copies: the column addresses are not shared with the loads
        // before the loop and held across it)
        int k_e = k;
        int64_t w_e = w;
        __asm__ volatile("" : "+v"(k_e));
        __asm__ volatile("" : "+v"(w_e));
        store_world_agent<N>(s, p, w_e * N + k_e, k_e);
        if (k_e == 0) store_world_shared<N>(s, p, w_e);
    }
}

template <int N, bool STORE = false>
__global__ __launch_bounds__(WAVE, 2) void k_rollout_shared(const Params p, const RolloutArgs r)
{
    if constexpr (SharedRollout<N>::value) {
        __shared__ typename SharedRollout<N>::Lds sm;
        const uint4 *g = (const uint4 *)&PIECE_CODE<N>;
        for (int i = (int)threadIdx.x; i < obs_width(N) / 4; i += WAVE) sm.code[i] = g[i];
        rollout_shared_world<N, typename SharedRollout<N>::Lds, STORE>(p, r, sm);
    }
}

// One lane per world.
template <int N, int MODE>
__device__ __forceinline__ void step_world_lanes(const Params &p, float *tile)
{
    using T = ObsTile<N>;
    const int lane = threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * WAVE;
    const int64_t w = w0 + lane;
    const bool active = w < p.num_worlds;

    World<N> s;
    Ctx c = make_ctx(p, w, true);
    trace_point<MODE>(p, 0);
    Orig<N> o;  // event-only words as loaded (store only on change)
    if (active) {
        load_world(s, p, w);
        capture(o, s);
        if constexpr (MODE == MODE_SKIP) step_world_pre_obs(s, c, EachAgent(), p.diag_skip, p.diag_dup);
        else if constexpr (MODE != MODE_IO && MODE != MODE_IO_OBS) step_world_pre_obs(s, c);
    }
    trace_point<MODE>(p, 7);
    trace_resets<MODE>(p, active, s);
    if (active) {
        // reward + state columns first, so their stores drain while the
        // observation rows are built
        if constexpr (MODE != MODE_IO && MODE != MODE_IO_OBS) sys_reward(s);
        store_world(s, p, w, &o);
    }
    trace_point<MODE>(p, 8);
    if constexpr (MODE == MODE_IO || MODE == MODE_NO_OBS) {
        return;
    } else if constexpr (MODE == MODE_DIRECT_OBS || !T::STAGED) {
        if (active) sys_fill_obs(s, c);
    } else {
        const int32_t ib = active ? inbounder_id(s) : -1;
        const bool share = active && obs_sharable(s);
        SharedObs<N> sh;
        if (share) shared_obs_prepare(s, c, sh);
#pragma unroll
        for (int a = 0; a < N; a++) {
            float *trow = tile + lane * T::RS;
            const bool fast = active && (share || canonical_slots(s, a));
            if (share) {
                RowSink o;
                o.row = trow; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
                emit_row_shared(s, c, sh, a, o, ib);
            } else if (fast) {
                fill_obs_fast(s, c, a, trow, ib);
            } else if (active) {
                fill_obs_slow(s, c, a, p.c.obs + (w * N + a) * (int64_t)obs_width(N), ib);
            }
            __syncthreads();
            flush_tile<N, T::QW, T::RS, 0, T::QW, N>(tile, p.c.obs, w0 * N + a, __ballot(fast), lane);
            __syncthreads();
        }
    }
    trace_point<MODE>(p, 9);
}

template <int N, bool LINES>
constexpr int tile_floats()
{
    if constexpr (Lanes<N>::SHARED) return BB_SHARED_TILE ? PhasedTile<N>::FLOATS : 4;
    return Lanes<N>::LPW == N ? StepTile<N, LINES>::FLOATS : ObsTile<N>::FLOATS;
}

#ifndef BB_STEP_MINW
#define BB_STEP_MINW 2  // waves per SIMD the register budget is sized for
#endif
// REC: the step also records agent rec_agent's rows into Params::rec_obs
// (PPO's per-step loop, N = 2; a separate instantiation, so the plain step
// carries none of it)
template <int N, int MODE, bool LINES = false, bool REC = false>
__global__ __launch_bounds__(WAVE, BB_STEP_MINW) void k_step(const Params p)
{
    __shared__ float4 tile4[tile_floats<N, LINES>() / 4];
    if constexpr (Lanes<N>::SHARED) {
        __shared__ SharedLds<N> sm;
        if constexpr (BB_OBS_PIECES && MODE != MODE_DIRECT_OBS && !SharedTiled<N>::value) {
            // the decode table into LDS (one copy per wave, L2-resident)
            const uint4 *g = (const uint4 *)&PIECE_CODE<N>;
            for (int i = (int)threadIdx.x; i < obs_width(N) / 4; i += WAVE) sm.code[i] = g[i];
        }
        step_shared_world<N, MODE, LINES>(p, (float *)tile4, sm, (int)blockIdx.x, (int)threadIdx.x);
    } else if constexpr (Lanes<N>::LPW == N) {
        step_agent_lanes<N, MODE, LINES, REC>(p, (float *)tile4, (int)blockIdx.x, (int)threadIdx.x);
    } else {
        step_world_lanes<N, MODE>(p, (float *)tile4);
    }
}

// k_step_loop<2>: `steps` steps of bb_step_n_staged in one launch.  Worlds
// are independent, so each wave runs its worlds' steps back to back -- step t
// reads the staged action rows t (actions + t * act_step), loads the state its
// own lanes stored at the end of step t - 1 and stores every column, the
// observation rows, rewards and done flags, exactly as k_step -- with no kernel
// boundary between steps: the waves drift apart and one's memory phases
// overlap another's systems (k_rollout_ppo's structure without the policy).
// Bit-identical to `steps` k_step launches (same code, same order per world).
// G > 1: workgroups of G waves kept in step by a barrier after every step
// (launch_step_loop_t picks G).

template <int N, bool LINES, int G>
__global__ __launch_bounds__(WAVE * G, BB_STEP_MINW) void k_step_loop(const Params p, int32_t *actions,
                                                                      int64_t act_step, int32_t steps)
{
    if constexpr (N == 2 && Lanes<N>::LPW == N && !Lanes<N>::SHARED) {
        constexpr int TF = tile_floats<N, LINES>();
        __shared__ float4 tile4[G * TF / 4];
        const int wave = G == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE);
        for (int32_t t = 0; t < steps; t++) {
            // opaque per-step copies of the indices (nothing derived from them
            // is computed before the loop and held across it)
            int32_t t_t = t, blk_t = (int)blockIdx.x * G + wave, lane_t = (int)threadIdx.x % WAVE;
            // (without these copies: 256 VGPRs + 350-400 B of scratch per lane)
            __asm__ volatile("" : "+s"(t_t), "+s"(blk_t));
            __asm__ volatile("" : "+v"(lane_t));
            Params pt = p;
            pt.c.action = actions + (int64_t)t_t * act_step;
            step_agent_lanes<N, MODE_FULL, LINES, false>(pt, (float *)tile4 + wave * TF, blk_t, lane_t);
            // this step's stores before the next step's loads (the wave's own
            // lanes' words; same wave, same vector L1); the tile is free again
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            if constexpr (G > 1) __syncthreads();
            else wave_sync();
        }
    } else if constexpr (Lanes<N>::SHARED && BB_OBS_PIECES && !SharedTiled<N>::value) {
        // N >= 4: the shared-LDS-world step (one wave per 64 / N worlds) the
        // same way, the row decode table loaded once per wave.  (With G > 1
        // the step's own workgroup barriers -- every one of them reached once
        // per step by every wave, whatever its worlds -- keep the G waves in
        // step.)
        constexpr int TF = tile_floats<N, LINES>();
        __shared__ float4 tile4[G * TF / 4];
        __shared__ SharedLds<N> sm[G];
        const int wave = G == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE);
        const uint4 *g = (const uint4 *)&PIECE_CODE<N>;
        for (int i = (int)(threadIdx.x % WAVE); i < obs_width(N) / 4; i += WAVE) sm[wave].code[i] = g[i];
        for (int32_t t = 0; t < steps; t++) {
            int32_t t_t = t, blk_t = (int)blockIdx.x * G + wave, lane_t = (int)(threadIdx.x % WAVE);
            __asm__ volatile("" : "+s"(t_t), "+s"(blk_t));
            __asm__ volatile("" : "+v"(lane_t));
            Params pt = p;
            pt.c.action = actions + (int64_t)t_t * act_step;
            step_shared_world<N, MODE_FULL, LINES>(pt, (float *)tile4 + wave * TF, sm[wave], blk_t, lane_t);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __syncthreads();
        }
    }
}

template <int N>
__global__ __launch_bounds__(256) void k_init(const Params p)
{
    const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= p.num_worlds) return;
    init_world<N>(p, w);
}

// ev0/ev1 (optional): hipExtLaunchKernel records the kernel's own start and
// end in them (the dispatch packet's timestamps, as rocprofv3 reports them).
// Whole-line observation passes once a step's state and rows no longer fit
// comfortably in the 256 MiB Infinity Cache (see StepTile).
constexpr int64_t LINES_MIN_BYTES = 192ll << 20;
// N >= 4: the rows and columns are stored non-temporally once a step's bytes
// exceed this.  Measured at 65 536 worlds: N = 4 (266 MB per step) 69.6 us
// plain vs 73.9 nt; N = 10 (1.28 GB) 343 vs 323.
constexpr int64_t SHARED_BEYOND_BYTES = 384ll << 20;
template <int N>
bool step_lines(int64_t num_worlds)
{
    const int64_t per_world = (int64_t)N * (obs_width(N) * 4 + 240) + 160;  // rows + state columns
    if constexpr (Lanes<N>::SHARED) return num_worlds * per_world > SHARED_BEYOND_BYTES;
    return Lanes<N>::LPW == N && num_worlds * per_world > LINES_MIN_BYTES;
}

// Compute units of the current device (256 on MI355X).
static unsigned device_cus()
{
    static const unsigned v = [] {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        return (unsigned)cus;
    }();
    return v;
}

// k_step_loop's workgroup size for a grid of `waves`.
static int step_loop_group(int64_t waves)
{
    // (49 152 worlds = 1.5 waves per SIMD: 4-wave workgroups leave half the CUs
    // with one workgroup and half with two, 18.1 us per step; 2-wave ones
    // spread evenly, 15.6)
    const int64_t cus = device_cus();
    if (waves < 4 * cus) return 1;
    return waves % (4 * cus) != 0 && waves % (2 * cus) == 0 ? 2 : 4;
}

template <int N>
hipError_t launch_step_loop_t(const Params &p, int32_t *actions, int32_t steps, hipStream_t s, hipEvent_t ev0,
                              hipEvent_t ev1)
{
    if constexpr (N == 2 && Lanes<N>::LPW == N && !Lanes<N>::SHARED) {
        // 4-wave workgroups in step (a barrier per step) while the grid still
        // gives every CU one; 1-wave workgroups drifting freely below that.
        // Measured (profiles/r05/x_, y_): 65 536 worlds 22.6 (1) / 19.6 (4) /
        // 20.3 (8) us per step against 21.3 with one k_step per step; 8 192
        // 6.6 (1) / 9.9 (4; 64 CUs busy); 262 144 64.0 / 61.7 / 66.9.
        const int64_t waves = (p.num_worlds + Lanes<N>::WPB - 1) / Lanes<N>::WPB;
        const int g = step_loop_group(waves);
        const dim3 grid((unsigned)((waves + g - 1) / g)), block(WAVE * g);
        const int64_t act_step = p.num_worlds * N * 6;
        const bool lines = step_lines<N>(p.num_worlds);
#define BB_LOOP(L, G) hipExtLaunchKernelGGL((k_step_loop<N, L, G>), grid, block, 0, s, ev0, ev1, 0, p, actions, act_step, steps)
        switch (g) {
        case 4: if (lines) BB_LOOP(true, 4); else BB_LOOP(false, 4); break;
        case 2: if (lines) BB_LOOP(true, 2); else BB_LOOP(false, 2); break;
        default: if (lines) BB_LOOP(true, 1); else BB_LOOP(false, 1); break;
        }
#undef BB_LOOP
        return hipGetLastError();
    } else if constexpr (Lanes<N>::SHARED && BB_OBS_PIECES && !SharedTiled<N>::value) {
        // (1-wave workgroups: 2 / 4 waves kept in step measured no faster --
        // 65 536 x 4 55.2 / 56.2 / 56.0 us per step, x 10 245.9 / 254.9 / 260.0,
        // profiles/r05/aj_shared_g.txt)
        constexpr int WPB = Lanes<N>::WPB;
        const dim3 grid((unsigned)((p.num_worlds + WPB - 1) / WPB)), block(WAVE);
        const int64_t act_step = p.num_worlds * N * 6;
#define BB_LOOP(L, G) hipExtLaunchKernelGGL((k_step_loop<N, L, G>), grid, block, 0, s, ev0, ev1, 0, p, actions, act_step, steps)
        if (step_lines<N>(p.num_worlds)) BB_LOOP(true, 1);
        else BB_LOOP(false, 1);
#undef BB_LOOP
        return hipGetLastError();
    } else {
        return hipErrorNotSupported;
    }
}

template <int N>
hipError_t launch_step_t(const Params &p, int mode, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1)
{
    constexpr int WPB = Lanes<N>::WPB;
    const dim3 grid((unsigned)((p.num_worlds + WPB - 1) / WPB)), block(WAVE);
#define BB_LAUNCH(m) hipExtLaunchKernelGGL(k_step<N, m>, grid, block, 0, s, ev0, ev1, 0, p)
    if (p.rec_obs && !(N == 2 && Lanes<N>::LPW == N && !Lanes<N>::SHARED))
        return hipErrorNotSupported;  // a record the step cannot write (step_records_t)
    if constexpr (N == 2 && Lanes<N>::LPW == N && !Lanes<N>::SHARED) {
        static_assert(obs_width(N) == POL_IN, "the record rows are the sim's rows");
        if (mode == MODE_FULL && p.rec_obs) {
            if (step_lines<N>(p.num_worlds)) hipExtLaunchKernelGGL((k_step<N, MODE_FULL, true, true>), grid, block, 0, s, ev0, ev1, 0, p);
            else hipExtLaunchKernelGGL((k_step<N, MODE_FULL, false, true>), grid, block, 0, s, ev0, ev1, 0, p);
            return hipGetLastError();
        }
    }
    switch (mode) {
    case MODE_FULL:
        if (step_lines<N>(p.num_worlds)) hipExtLaunchKernelGGL(k_step<N, MODE_FULL, true>, grid, block, 0, s, ev0, ev1, 0, p);
        else hipExtLaunchKernelGGL(k_step<N, MODE_FULL>, grid, block, 0, s, ev0, ev1, 0, p);
        break;
    case MODE_IO: BB_LAUNCH(MODE_IO); break;
    case MODE_IO_OBS: BB_LAUNCH(MODE_IO_OBS); break;
    case MODE_DIRECT_OBS: BB_LAUNCH(MODE_DIRECT_OBS); break;
    case MODE_NO_OBS: BB_LAUNCH(MODE_NO_OBS); break;
    case MODE_SKIP: BB_LAUNCH(MODE_SKIP); break;
    case MODE_TRACE: BB_LAUNCH(MODE_TRACE); break;
    default: return hipErrorInvalidValue;
    }
#undef BB_LAUNCH
    return hipGetLastError();
}

// The whole-register-file rollout while the grid fits one wave per SIMD (every
// CU of the device, 4 SIMDs each); DIAG_ROLLOUT_MINW = 1 / 2 forces it (tests).
static bool rollout_minw1(unsigned waves)
{
    const int forced = diag_or(DIAG_ROLLOUT_MINW, 0);
    if (forced) return forced == 1;
    return waves <= 4u * device_cus();
}

// k_rollout_split while its workgroups (2 waves) fit one wave per SIMD: at
// most 2 per CU.  DIAG_ROLLOUT_SPLIT forces it off / on (tests).
#ifndef BB_ROLLOUT_SPLIT
#define BB_ROLLOUT_SPLIT 1
#endif
static bool rollout_split(unsigned groups)
{
    const int forced = diag_or(DIAG_ROLLOUT_SPLIT, -1);
    if (forced >= 0) return forced != 0;
    return BB_ROLLOUT_SPLIT != 0 && groups <= 2u * device_cus();
}

// The K-step rollout kernel a grid of num_worlds takes (RolloutKernel); the
// launcher and the name query (bench.py's kernel names) use this one rule.
template <int N>
int rollout_kernel_t(int64_t num_worlds)
{
    if constexpr (SharedRollout<N>::value) {
        return RK_SHARED;
    } else if constexpr (!FusedRollout<N>::value) {
        return RK_NONE;
    } else {
        const unsigned grid = (unsigned)((num_worlds + Lanes<N>::WPB - 1) / Lanes<N>::WPB);
        return rollout_split(grid) ? RK_SPLIT : rollout_minw1(grid) ? RK_MINW1 : RK_MINW2;
    }
}

template <int N>
hipError_t launch_rollout_t(const Params &p, const RolloutArgs &r, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1)
{
    constexpr int WPB = Lanes<N>::WPB;
    const dim3 grid((unsigned)((p.num_worlds + WPB - 1) / WPB)), block(WAVE);
    if (r.store_state && (r.reward != p.c.reward || r.done != p.c.done || r.rd_step != 0))
        return hipErrorInvalidValue;  // the resident loop stores reward / done with the state
    const int kind = rollout_kernel_t<N>(p.num_worlds);
    if constexpr (SharedRollout<N>::value) {
        // (the resident instance only while the step fits the Infinity Cache,
        // bb::resident_staged: beyond it the reloading loop is faster)
        if (r.store_state && step_lines<N>(p.num_worlds)) return hipErrorNotSupported;
        if (r.store_state)
            hipExtLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_shared<N, true>), grid, block, 0, s, ev0, ev1, 0, p, r);
        else
            hipExtLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_shared<N>), grid, block, 0, s, ev0, ev1, 0, p, r);
        return hipGetLastError();
    } else if constexpr (!FusedRollout<N>::value) {
        return hipErrorNotSupported;
    } else {
        switch (kind) {
        case RK_SPLIT:
            if (r.store_state)
                hipExtLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_split<N, true>), grid, dim3(2 * WAVE), 0, s, ev0, ev1, 0, p, r);
            else
                hipExtLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_split<N>), grid, dim3(2 * WAVE), 0, s, ev0, ev1, 0, p, r);
            break;
        case RK_MINW1:
            if (r.store_state)
                hipExtLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout<N, 1, 1, true>), grid, block, 0, s, ev0, ev1, 0, p, r);
            else
                hipExtLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout<N, 1>), grid, block, 0, s, ev0, ev1, 0, p, r);
            break;
        default:
            if (r.store_state)
                hipExtLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout<N, 2, 1, true>), grid, block, 0, s, ev0, ev1, 0, p, r);
            else
                hipExtLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout<N, 2>), grid, block, 0, s, ev0, ev1, 0, p, r);
            break;
        }
        return hipGetLastError();
    }
}

template <int N>
hipError_t launch_rollout_policy_t(const Params &p, const PolicyRolloutArgs &r, hipStream_t s)
{
    if constexpr (N != 2 || !FusedRollout<N>::value) {
        return hipErrorNotSupported;
    } else {
        // 2 policy waves (3 waves per workgroup: each its own SIMD, the sim
        // wave with the SIMD's whole register file, no spill).  4 (5 waves:
        // two share a SIMD, the 256-register budget, 45 spilled VGPRs)
        // measured ahead at 8 192 worlds in round 5 (9.66 ->
        // 9.48 us per step, profiles/r05/ad_pw_ab.txt) and behind in round 6
        // (9.80 vs 9.62, three interleaved pairs, profiles/r06/o_ppo_pw_ab.txt;
        // per call 22.3 + 8.99 us per step vs 18.9 + 8.84); 16 384: 18.2 vs 12.1.
        // DIAG_PPO_PWAVES = 2 / 4 forces it (tests).
        const dim3 grid((unsigned)((p.num_worlds + 31) / 32));
        const int forced = diag_or(DIAG_PPO_PWAVES, 0);
        const int pw = forced == 2 || forced == 4 ? forced : 2;
        if (pw == 4)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_policy<N, 2, 4>), grid, dim3(WAVE * 5), 0, s, p, r);
        else if (grid.x <= device_cus())
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_policy<N, 1, 2>), grid, dim3(WAVE * 3), 0, s, p, r);
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_policy<N, 2, 2>), grid, dim3(WAVE * 3), 0, s, p, r);
        return hipGetLastError();
    }
}

#if BB_N == 2
// k_rollout_ppo / k_step_ppo: 8-wave workgroups (the weights' 32.6 KB shared
// by 256 worlds, 155 KB of LDS: one workgroup and 2 waves per SIMD per CU)
// while the grid fills the device with them, 4-wave workgroups below that.
hipError_t launch_rollout_ppo_2(const Params &p, const PpoStepArgs &a, int32_t steps, hipStream_t s)
{
    const int64_t waves = (p.num_worlds + WAVE / 2 - 1) / (WAVE / 2);
    const int64_t cus = device_cus();
    // the largest workgroup whose grid still gives every CU one
    const int wpg = waves >= 8 * cus ? 8 : waves >= 4 * cus ? 4 : waves >= 2 * cus ? 2 : 1;
    const dim3 grid((unsigned)((waves + wpg - 1) / wpg)), block(WAVE * wpg);
    if (steps < 1) return hipSuccess;
    switch (wpg) {
    case 8: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_ppo<8>), grid, block, 0, s, p, a, steps); break;
    case 4: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_ppo<4>), grid, block, 0, s, p, a, steps); break;
    case 2: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_ppo<2>), grid, block, 0, s, p, a, steps); break;
    default: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rollout_ppo<1>), grid, block, 0, s, p, a, steps); break;
    }
    return hipGetLastError();
}

hipError_t launch_step_ppo_2(const Params &p, const PpoStepArgs &a, hipStream_t s)
{
    const int64_t waves = (p.num_worlds + WAVE / 2 - 1) / (WAVE / 2);
    const bool big = waves >= 8 * (int64_t)device_cus();
    const int wpg = big ? 8 : 4;
    const dim3 grid((unsigned)((waves + wpg - 1) / wpg)), block(WAVE * wpg);
    if (big) {
        if (a.last) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step_ppo<8, true>), grid, block, 0, s, p, a);
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step_ppo<8, false>), grid, block, 0, s, p, a);
    } else {
        if (a.last) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step_ppo<4, true>), grid, block, 0, s, p, a);
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step_ppo<4, false>), grid, block, 0, s, p, a);
    }
    return hipGetLastError();
}
#endif

template <int N>
hipError_t launch_init_t(const Params &p, hipStream_t s)
{
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_init<N>), dim3((unsigned)((p.num_worlds + 255) / 256)), dim3(256), 0, s, p);
    return hipGetLastError();
}

template hipError_t launch_step_t<BB_N>(const Params &, int, hipStream_t, hipEvent_t, hipEvent_t);
template hipError_t launch_step_loop_t<BB_N>(const Params &, int32_t *, int32_t, hipStream_t, hipEvent_t, hipEvent_t);
template hipError_t launch_init_t<BB_N>(const Params &, hipStream_t);
template hipError_t launch_rollout_t<BB_N>(const Params &, const RolloutArgs &, hipStream_t, hipEvent_t, hipEvent_t);
template int rollout_kernel_t<BB_N>(int64_t);
template hipError_t launch_rollout_policy_t<BB_N>(const Params &, const PolicyRolloutArgs &, hipStream_t);
template <> bool fused_rollout<BB_N>() { return FusedRollout<BB_N>::value || SharedRollout<BB_N>::value; }
template <> bool step_records_t<BB_N>() { return BB_N == 2 && Lanes<BB_N>::LPW == BB_N && !Lanes<BB_N>::SHARED; }
// At 2 agents always; the shared-world kernel while the step stays in the
// Infinity Cache (65 536 x 4 52.4 -> 48.3 us per step; beyond it the
// reloading loop is faster, 131 072 x 4 96.3 vs 114.7; profiles/r05/ar_sweep.txt).
template <> bool resident_staged<BB_N>(int64_t num_worlds)
{
    if constexpr (FusedRollout<BB_N>::value) return true;
    else if constexpr (SharedRollout<BB_N>::value) return !step_lines<BB_N>(num_worlds);
    else return false;
}
template <> int step_grid<BB_N>(int64_t num_worlds)
{
    return (int)((num_worlds + Lanes<BB_N>::WPB - 1) / Lanes<BB_N>::WPB);  // waves of the MODE_FULL launch
}

}  // namespace bb
