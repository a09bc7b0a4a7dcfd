// mrp_world.h -- one MultiRobotPuzzle world ("lane") stepped by one wavefront.
//
// This is the MI355X-native restatement of the per-timestep path of
// gym_puzzles/envs/multi_robot_puzzle_00.py:413-521 (v0) and multi_robot_puzzle_02.py:444-584
// (v2): action -> forces, the Box2D v2.3 world.Step(1/50, 180, 60) (broad phase, polygon SAT,
// sequential-impulse contact solver with the 2-point block solver, position solver, TOI),
// then contact flags, distances, observation, reward, done.
//
// Execution model: one 64-thread workgroup (one wave) owns one lane for a whole k_step.  The
// lane's persistent state (LaneState<ENV>, a POD of 32-bit words) is stored lane-major in HBM --
// each lane one contiguous block, moved by the wave as coalesced 16-B granules (mrp_lane.h
// StateIO) -- and lives in LDS (Shared<ENV>) for the step.  Thread 0 runs the order-sensitive
// serial parts (tree reinsertions, sorted AddPair, contact commit and events, island set-up, TOI
// bookkeeping); all 64 threads run the data-parallel parts (pair tests, one contact's SAT per
// thread, the island DFS, the fixtures' swept AABBs, TOI candidate scans, state I/O); the velocity and position iterations run on the whole
// wave with the island in registers (one or two contacts: every thread evaluates the same update)
// or spread across the wave (larger islands: contact i's constants in thread i, body k's state in
// thread k, one contact update after the other through v_readlane / v_writelane).
//
// Box2D's pointer-linked lists become index lists: the world contact list is a doubly
// linked list of slots in creation-descending order, and a body's contact-edge list is the
// world list filtered by that body (same relative order, since both are head-inserted at
// contact creation).  The dynamic AABB tree is kept node-for-node (same allocation order,
// SAH insertion, rotations) because its free list decides the proxy ids after a reset, and
// proxy ids decide fixture A/B roles and the contact (= Gauss-Seidel) order.
#pragma once
#include <type_traits>

#include "mrp_config.h"

namespace mrp {

constexpr int NULLN = -1;

// MRP_SOLVE_NOINLINE_LANES (build.py: the 3-block unit): the lanes-path sweep / pass loops as functions
// of their own (one call per island solve), so the machine scheduler treats each loop as it does in a
// small kernel (profiles/r3g_ab_scheduler.txt).  Every other loop is inlined into k_step.
#define MRP_SOLVE_FN __device__ __forceinline__
#ifdef MRP_SOLVE_NOINLINE_LANES
#define MRP_LANES_FN __device__ __attribute__((noinline))
#else
#define MRP_LANES_FN MRP_SOLVE_FN
#endif
// Per-unit compile choices (build.py UNIT_FLAGS; each measured per config):
// MRP_LANES_PAIRS=1   the lanes-path sweeps two per loop trip (v0, v3)
// MRP_VEL_PICK2=1     the block solver's case tests as two ballots of the compares (no bool in a VGPR)
// MRP_VEL_VTCROSS=1   the tangent speed b2Dot(dv, (n.y, -n.x)) as dv.x*n.y - dv.y*n.x (pcross: a + (-b) is
//                     a - b exactly), so the tangent is never materialised for it
// MRP_VEL_BFREE=1     the block solver's four cases evaluated together and picked by per-lane selects
//                     (no chain of case tests, no ballot -> branch); MRP_VEL_BFREE_LANES=1 restricts it to
//                     the lanes path (3+ contacts)
// MRP_FRESH_REGS=1    values k_step needs late in the step are made where they are used, and the thread id
//                     is made opaque per island and TOI pass (refresh_tid) (v0, v3)
// Diagnostic builds (never shipped): MRP_STAMPS (+ MRP_STAMPS_TOI) per-phase timing, MRP_PROGRESS
// hang localisation.  The arms measured and dropped in rounds 3-5 are kept as patches under
// profiles/ (r6_dropped_arms.patch), not in this header.
#ifndef MRP_LANES_PAIRS
#define MRP_LANES_PAIRS 0
#endif
#ifndef MRP_VEL_PICK2
#define MRP_VEL_PICK2 0
#endif
#ifndef MRP_VEL_VTCROSS
#define MRP_VEL_VTCROSS 0
#endif
#ifndef MRP_VEL_BFREE
#define MRP_VEL_BFREE 0
#endif
#ifndef MRP_VEL_BFREE_LANES
#define MRP_VEL_BFREE_LANES 0
#endif
#ifndef MRP_FRESH_REGS
#define MRP_FRESH_REGS 0
#endif
#if MRP_VEL_VTCROSS
#define MRP_VT(dv, n, t) pcross(dv, n)
// lambda * (n.y, -n.x) = (lambda*n.y, -(lambda*n.x)) exactly: a swapped product with its high half negated
#define MRP_PT(l, n, t) ([](const P2 q_) { return p2(q_.x, -q_.y); }(pbc(l) * (n).yx))
#else
#define MRP_VT(dv, n, t) pdot(dv, t)
#define MRP_PT(l, n, t) (pbc(l) * (t))
#endif

// v_writelane_b32 (clang exposes no builtin for it; the LLVM intrinsic is bound by name, so the
// compiler still inserts the readlane -> writelane wait states itself)
extern "C" __device__ int mrp_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

// Diagnostic phase timing (build with -DMRP_STAMPS; never in the shipped build): thread 0 of
// every lane accumulates s_memtime deltas per phase in LDS and writes its trace row to g_trace
// with plain stores at the end of its step; k_stamp_fold (mrp_lane.h) folds the rows into the
// totals after the launch, so k_step issues no global atomics.
#ifdef MRP_STAMPS
static __device__ unsigned long long g_stamps[16];     // per-phase sums over lane-steps
static __device__ unsigned long long g_pmax[16];       // per-phase max over lane-steps
static __device__ unsigned long long g_stepmax[256];   // per step (stepCounter mod 256): slowest lane's total
static __device__ unsigned long long g_rt[2];          // sums of lane totals: s_memtime ticks, s_memrealtime ticks
constexpr int MRP_TRACE_W = 40;   // include/mrp.h MRP_TRACE_WORDS (static_assert in mrp_lane.h)
static __device__ uint32_t g_trace[16384][MRP_TRACE_W];   // last step per lane: phases 0-10, total, nc, toi, pos, vel-units,
                                                       // velocity / position / island-set-up cycles, largest island,
                                                       // 20/21 TOI split (candidate scan + b2TimeOfImpact, events),
                                                       // 22/23 collide split (narrow phase, serial commit), 24-26 load
                                                       // sub-phases (state, tables, barrier), 27 step index mod 256,
                                                       // 28/29 s_memrealtime at entry / end, 30/31 HW_ID / XCC_ID,
                                                       // 32 island building (DFS), 33 island write-back and
                                                       // integration (island_mid / island_post), 34 fixture
                                                       // synchronisation after the solve, 35 the TOI scan alone
#define MRP_NOW() __builtin_amdgcn_s_memtime()
#define MRP_SUB(k, t0) do { if (tid == 0) sh.trace[k] += (uint32_t)(__builtin_amdgcn_s_memtime() - (t0)); } while (0)
#define MRP_TRACE(k, v) do { if (tid == 0) sh.trace[k] += (v); } while (0)
#define MRP_STAMP(k)                                                                        \
    do {                                                                                    \
        if (tid == 0) {                                                                     \
            unsigned long long _t = __builtin_amdgcn_s_memtime();                           \
            sh.trace[k] += (uint32_t)(_t - sh.stamp_t);                                     \
            sh.stamp_t = _t;                                                                \
        }                                                                                   \
    } while (0)
#else
#define MRP_STAMP(k) MRP_PROG(0x100u * ((k) + 1))
#define MRP_TRACE(k, v) do {} while (0)
#define MRP_NOW() 0ull
#define MRP_SUB(k, t0) do { (void)(t0); } while (0)
#endif
// Diagnostic hang localisation (build with -DMRP_PROGRESS; never in the shipped build): thread 0
// of every lane stores the last progress point it reached into host-mapped memory, which a host
// watchdog reads while a launch is still running (tools/hang_probe.py).
#ifdef MRP_PROGRESS
static __device__ uint32_t* g_progress;
#define MRP_PROG(k)                                                                                          \
    do {                                                                                                     \
        if (threadIdx.x == 0 && g_progress)                                                                  \
            __hip_atomic_store(g_progress + blockIdx.x, (uint32_t)(k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
    } while (0)
#else
#define MRP_PROG(k) do {} while (0)
#endif
// Loop guards: every loop whose trip count depends on lane data has a bound no valid world can
// reach; a guard that trips records its code in LaneState::fault and leaves the loop, so a
// corrupted lane finishes its step (and is reported by mrp_get_faults) instead of hanging the GPU.
constexpr int MRP_FAULT_TREE_UP = 1, MRP_FAULT_TREE_DOWN = 2, MRP_FAULT_TREE_REMOVE = 3, MRP_FAULT_CONTACT_LIST = 4,
              MRP_FAULT_ISLANDS = 5, MRP_FAULT_TOI_PASSES = 6, MRP_FAULT_PAIR_DECODE = 7, MRP_FAULT_DFS = 8;
// Pool guards: the fixed per-lane pools (tree nodes, contact slots, move buffer, island arrays) are
// sized from the configs' geometry and never fill in a valid world (tests/test_oracle.py checks the
// oracle's high-water marks against them); a full pool records its code and the insertion is
// skipped, so no index ever leaves its array.
constexpr int MRP_FAULT_TREE_POOL = 9, MRP_FAULT_CONTACT_POOL = 10, MRP_FAULT_MOVE_BUFFER = 11, MRP_FAULT_ISLAND_POOL = 12;
constexpr float LINEAR_SLOP = 0.005f;
constexpr float AABB_EXT = 0.1f;
constexpr float AABB_MUL = 2.0f;
constexpr float MAX_TRANSLATION = 2.0f;
constexpr float MAX_TRANSLATION_SQ = MAX_TRANSLATION * MAX_TRANSLATION;
constexpr float B2_PI = 3.14159265359f;
constexpr float MAX_ROTATION = 0.5f * B2_PI;
constexpr float MAX_ROTATION_SQ = MAX_ROTATION * MAX_ROTATION;
constexpr float BAUMGARTE = 0.2f;
constexpr float TOI_BAUMGARTE = 0.75f;
constexpr float VELOCITY_THRESHOLD = 1.0f;
constexpr float MAX_LINEAR_CORRECTION = 0.2f;
constexpr int MAX_SUBSTEPS = 8;
constexpr int MAX_TOI_CONTACTS = 32;
constexpr float FLT_EPS = 1.1920928955078125e-7f;
constexpr float FLT_MAXV = 3.40282346638528859811704183484516925e+38f;

// contact flags (b2Contact)
constexpr int CF_ISLAND = 1, CF_TOUCHING = 2, CF_ENABLED = 4, CF_TOI = 32;
constexpr int MT_FACEA = 1, MT_FACEB = 2;

template <int ENV> struct alignas(16) LaneState {   // 16-B granules: moved with dwordx4 per thread
    using D = Dims<ENV>;
    static constexpr int ND = D::NA + D::NB;
    static constexpr int C = D::CMAX;
    static constexpr int TN = tree_n<ENV>();
    static constexpr int MOVE_N = move_n<ENV>();
    using PMask = typename std::conditional<(TN <= 32), uint32_t, uint64_t>::type;   // one bit per proxy (tree node) id
    static_assert(D::NF < MOVE_N, "move buffer smaller than the proxy count");
    static_assert(D::NA + D::NB + 4 <= MAXBODY && D::NF <= MAXF, "env tables too small for this env id");
    // dynamic bodies (blocks, then agents): transform, sweep, velocity, force accumulators
    float xpx[ND], xpy[ND], xs[ND], xc[ND];
    float c0x[ND], c0y[ND], cx[ND], cy[ND], a0[ND], a[ND], alpha0[ND];
    float vx[ND], vy[ND], w[ND];
    float fx[ND], fy[ND], tq[ND];
    // fixtures -> broad-phase proxy id
    int proxy[D::NF];
    // dynamic AABB tree (fat AABBs)
    float tlx[TN], tly[TN], thx[TN], thy[TN];
    int tpar[TN], tc1[TN], tc2[TN], th[TN], tud[TN];
    int root, freeList, nodeCount, moveCount;
    int moveBuf[MOVE_N];
    // contacts (slot pool + creation-descending doubly linked list)
    // cHW: every slot >= cHW holds its initial contents (zero, cnext[c] = c + 1): slots are taken
    // from the head of the free list, which after a reset is 0, 1, 2, ... and to which freed slots
    // return at the head, so the never-used slots stay an ordered tail.  k_step moves only slots
    // < cHW between HBM and LDS (NCA arrays from cnext on), and a reset zeroes slots < cHW.
    int cHead, cFree, cCount, cHW;
    static constexpr int NCA = 24;   // contact arrays cnext .. mid[1], C words each, contiguous
    int cnext[C], cprev[C], cfa[C], cfb[C], cflags[C], ctoiCount[C];
    float ctoi[C], cfric[C];
    int mpc[C], mtype[C];
    float mlnx[C], mlny[C], mlpx[C], mlpy[C];
    float mpx[2][C], mpy[2][C], mni[2][C], mti[2][C];
    uint32_t mid[2][C];
    // world
    float inv_dt0;
    int newFixture, haveBodies, episode;
    uint32_t stepCounter;
    int elapsed, blks_in_place, prev_blks_in_place;
    int goal_contact[D::NA];
    int wall_contact;
    int fault;   // 0, or the MRP_FAULT_* code of a loop guard that tripped (no step may spin forever)
    double agent_dist[D::NA];
    double block_distance[D::NB];
    double goal[D::NB][3];
    long long toiEvents, posIters;
    long long touching;    // touching contacts after each world.Step's Collide, summed (SURVEY.md 5 metrics)
    long long nonfinite;   // steps whose observation or body state held a NaN / inf
};

template <int ENV> constexpr int lane_words() { return (int)(sizeof(LaneState<ENV>) / 4); }

struct TOIOut { int state; float t; };

struct ClipV { V2 v; uint32_t id; };
struct VC {
    float rAx[2], rAy[2], rBx[2], rBy[2], ni[2], ti[2], nmass[2], tmass[2], vbias[2];
    float nx, ny, nm0, nm1, nm3, k0, k1, k3;   // K and K^-1 are symmetric: k2 == k1, nm2 == nm1 (not stored)
    float mA, mB, iA, iB, friction;
    int iaI, ibI, pointCount, slot;
};
struct PC {   // position constraint; body indices and mass data are read from the contact's VC
    float lpx[2], lpy[2], lnx, lny, lpx0, lpy0;
    float lcAx, lcAy, lcBx, lcBy, rA, rB;
    int type, pointCount;
};
template <int NBODY, int C> struct IslT {
    int bodies[NBODY];
    int contacts[C];
    float pcx[NBODY], pcy[NBODY], pa[NBODY], vvx[NBODY], vvy[NBODY], vw[NBODY];
    int nb, nc;
    int index[NBODY];   // body -> island index
};
struct SweepV { float lcx, lcy, c0x, c0y, cx, cy, a0, a, alpha0; };
struct DProxy { const V2* v; int count; float radius; };
struct SVert { V2 wA, wB, w; float a; int iA, iB; };
struct Simplex { SVert v0, v1, v2; int count; };
struct SCache { float metric; int count; int iA0, iA1, iA2, iB0, iB1, iB2; };
struct SepFn { int type; V2 lp, axis; };

// Per-launch LDS copy of the env tables the step indexes with lane-varying indices (fixture
// shapes, fixture -> body, per-body mass and damping, wall poses).  From __constant__ memory
// those reads are vector-memory loads whose divergent addresses serialise in the texture path
// (the parallel narrow phase and TOI give every thread its own contact); from LDS they are
// ds_read at LDS latency.
template <int ENV> struct LdsTables {
    static constexpr int NF = Dims<ENV>::NF, NBODY = Dims<ENV>::NA + Dims<ENV>::NB + 4;
    ShapeDef shape[NF];
    int fix_body[NF];
    float fix_friction[NF], fix_restitution[NF];
    float invMass[NBODY], invI[NBODY], lcx[NBODY], lcy[NBODY], linDamp[NBODY], angDamp[NBODY];
    int body_fix0[NBODY], body_nfix[NBODY];
    float wall_px[4], wall_py[4];
};

// Per-lane LDS working set of the cooperative (one wave per world) step.
template <int ENV> struct Shared {
    using D = Dims<ENV>;
    using LS = LaneState<ENV>;
    static constexpr int ND = LS::ND, NBODY = ND + 4, C = D::CMAX;
    LS S;
    LdsTables<ENV> lt;
    IslT<NBODY, C> isl;
    int hw_io;   // LaneState::cHW as k_step loaded it (its store writes slots < max(hw_io, cHW) back)
    float salpha0[4];
    // collide: contact list snapshot (the per-contact manifolds live in the phase union below)
    int clist[C];
    int ccount;
    uint8_t cover[C];
    // serial manifold slot (contact_update outside the parallel narrow phase)
    int spc, stype;
    float slnx, slny, slpx, slpy, spx[2], spy[2];
    uint32_t smid[2];
    // broad phase: active proxy ids (ascending)
    int nprox;
    typename LS::PMask moved;
    int prox[LS::TN];
    // TOI scan bookkeeping
    int tn, np, toi_done, toi_fnc, toi_solve;
    float toi_dt;
    int toiIA, toiIB;     // island indices of the TOI pair (position iterations)
    int tcand[C];
    int plan[C];          // per list position: -2 cached, >= 0 candidate index
    int pslot[C];
    // Phase-exclusive scratch (one member live at a time): island solver constraints,
    // narrow-phase manifolds, pair-overlap flags, TOI candidate sweeps/results.  Each is
    // consumed before the next phase writes another, which keeps a v0 lane in < 10 KB of LDS
    // (16 worlds per CU).
    union U {
        struct { VC vcs[C]; PC pcs[C]; } sol;
        struct {
            int tpc[C], ttype[C];
            float tlnx[C], tlny[C], tlpx[C], tlpy[C];
            float tpx[2][C], tpy[2][C];
            uint32_t tmid[2][C];
        } col;
        uint8_t pover[LS::TN * (LS::TN - 1) / 2];
        struct { SweepV tsA[C], tsB[C]; TOIOut tout[C]; } toi;
        struct { float lx[D::NF], ly[D::NF], hx[D::NF], hy[D::NF], dx[D::NF], dy[D::NF]; } fsync;   // solve_coop's end
    } u;
    // env I/O
    float obs[D::OBS];
    double reward;
    int done, kind;
    float act[D::ACT];
    double draws[D::NDRAW];
    unsigned long long stamp_t, stamp_t0, stamp_rt0;
#ifdef MRP_STAMPS
    uint32_t trace[MRP_TRACE_W];
#endif
};

template <int ENV> struct World {
    using D = Dims<ENV>;
    using LS = LaneState<ENV>;
    static constexpr int NA = D::NA, NB = D::NB, ND = LS::ND, NBODY = ND + 4, NF = D::NF, C = D::CMAX;

    using SH = Shared<ENV>;
    using Isl = IslT<NBODY, C>;
    SH& sh;
    LS& S;
    const LdsTables<ENV>& L;
    const EnvTables& T;
    const EnvParams& P;
    int tid;             // made opaque per island / TOI pass by refresh_tid (MRP_FRESH_REGS)
    int step_prio = 0;   // issue priority of this lane for the rest of the step (wave-uniform)
    int prio_floor = 0;  // lower bound for step_prio (k_step: from the lane's previous-step cost)

    __device__ __forceinline__ World(SH& s, const EnvTables& t, const EnvParams& p, int thread) : sh(s), S(s.S), L(s.lt), T(t), P(p), tid(thread) {}

    // MRP_FRESH_REGS: a copy of tid the compiler cannot prove equal to the one before it, so the LDS
    // addresses derived from it are made inside the loop that refreshes it, not hoisted to k_step's
    // entry and kept (or spilled) across the whole step
    __device__ __forceinline__ void refresh_tid() {
#if MRP_FRESH_REGS
        asm volatile("" : "+v"(tid));
#endif
    }

    // ------------------------------------------------------------------ bodies
    __device__ __forceinline__ bool is_dyn(int b) const { return b < ND; }
    __device__ __forceinline__ Xf xf(int b) const {
        Xf r;
        if (b < ND) { r.p = v2(S.xpx[b], S.xpy[b]); r.q.s = S.xs[b]; r.q.c = S.xc[b]; }
        else { r.p = v2(L.wall_px[b - ND], L.wall_py[b - ND]); r.q.s = 0.0f; r.q.c = 1.0f; }
        return r;
    }
    __device__ __forceinline__ V2 center(int b) const { return b < ND ? v2(S.cx[b], S.cy[b]) : v2(L.wall_px[b - ND], L.wall_py[b - ND]); }
    __device__ __forceinline__ V2 lc(int b) const { return v2(L.lcx[b], L.lcy[b]); }
    __device__ __forceinline__ void sync_transform(int b) {   // b2Body::SynchronizeTransform
        Rot q = rot_z(S.a[b]);
        S.xs[b] = q.s; S.xc[b] = q.c;
        V2 p = vsub(v2(S.cx[b], S.cy[b]), mul_rv(q, lc(b)));
        S.xpx[b] = p.x; S.xpy[b] = p.y;
    }

    // ------------------------------------------------------------------ dynamic tree
    __device__ __forceinline__ static float perim(float lx, float ly, float hx, float hy) { float wx = hx - lx; float wy = hy - ly; return 2.0f * (wx + wy); }
    __device__ __forceinline__ int t_alloc() {
        int id = S.freeList;
        if ((unsigned)id >= (unsigned)LS::TN) { S.fault = MRP_FAULT_TREE_POOL; id = LS::TN - 1; }   // never in a valid world
        S.freeList = S.tpar[id];
        S.tpar[id] = NULLN; S.tc1[id] = NULLN; S.tc2[id] = NULLN; S.th[id] = 0; S.tud[id] = -1;
        ++S.nodeCount;
        return id;
    }
    __device__ __forceinline__ void t_free(int id) { S.tpar[id] = S.freeList; S.th[id] = -1; S.tud[id] = -1; S.freeList = id; --S.nodeCount; }
    __device__ __forceinline__ bool t_leaf(int id) const { return S.tc1[id] == NULLN; }
    // contact-list walk guard: a list holds at most C contacts
    __device__ __forceinline__ bool list_ok(int& g) {
        if (++g <= C) return true;
        S.fault = MRP_FAULT_CONTACT_LIST;
        return false;
    }
    __device__ __forceinline__ void t_combine_into(int dst, int a, int b) {
        S.tlx[dst] = fmin_(S.tlx[a], S.tlx[b]); S.tly[dst] = fmin_(S.tly[a], S.tly[b]);
        S.thx[dst] = fmax_(S.thx[a], S.thx[b]); S.thy[dst] = fmax_(S.thy[a], S.thy[b]);
    }
    __device__ __forceinline__ int t_balance(int iA) {
        if (t_leaf(iA) || S.th[iA] < 2) return iA;
        int iB = S.tc1[iA], iC = S.tc2[iA];
        int balance = S.th[iC] - S.th[iB];
        if (balance > 1) {
            int iF = S.tc1[iC], iG = S.tc2[iC];
            S.tc1[iC] = iA; S.tpar[iC] = S.tpar[iA]; S.tpar[iA] = iC;
            int cp = S.tpar[iC];
            if (cp != NULLN) { if (S.tc1[cp] == iA) S.tc1[cp] = iC; else S.tc2[cp] = iC; }
            else S.root = iC;
            if (S.th[iF] > S.th[iG]) {
                S.tc2[iC] = iF; S.tc2[iA] = iG; S.tpar[iG] = iA;
                t_combine_into(iA, iB, iG); t_combine_into(iC, iA, iF);
                S.th[iA] = 1 + max(S.th[iB], S.th[iG]); S.th[iC] = 1 + max(S.th[iA], S.th[iF]);
            } else {
                S.tc2[iC] = iG; S.tc2[iA] = iF; S.tpar[iF] = iA;
                t_combine_into(iA, iB, iF); t_combine_into(iC, iA, iG);
                S.th[iA] = 1 + max(S.th[iB], S.th[iF]); S.th[iC] = 1 + max(S.th[iA], S.th[iG]);
            }
            return iC;
        }
        if (balance < -1) {
            int iD = S.tc1[iB], iE = S.tc2[iB];
            S.tc1[iB] = iA; S.tpar[iB] = S.tpar[iA]; S.tpar[iA] = iB;
            int bp = S.tpar[iB];
            if (bp != NULLN) { if (S.tc1[bp] == iA) S.tc1[bp] = iB; else S.tc2[bp] = iB; }
            else S.root = iB;
            if (S.th[iD] > S.th[iE]) {
                S.tc2[iB] = iD; S.tc1[iA] = iE; S.tpar[iE] = iA;
                t_combine_into(iA, iC, iE); t_combine_into(iB, iA, iD);
                S.th[iA] = 1 + max(S.th[iC], S.th[iE]); S.th[iB] = 1 + max(S.th[iA], S.th[iD]);
            } else {
                S.tc2[iB] = iE; S.tc1[iA] = iD; S.tpar[iD] = iA;
                t_combine_into(iA, iC, iD); t_combine_into(iB, iA, iE);
                S.th[iA] = 1 + max(S.th[iC], S.th[iD]); S.th[iB] = 1 + max(S.th[iA], S.th[iE]);
            }
            return iB;
        }
        return iA;
    }
    __device__ __forceinline__ void t_fix_upwards(int index) {
        for (int g = 0; index != NULLN; ++g) {
            if (g > LS::TN) { S.fault = MRP_FAULT_TREE_UP; break; }
            index = t_balance(index);
            int c1 = S.tc1[index], c2 = S.tc2[index];
            S.th[index] = 1 + max(S.th[c1], S.th[c2]);
            t_combine_into(index, c1, c2);
            index = S.tpar[index];
        }
    }
    __device__ __forceinline__ void t_insert(int leaf) {
        if (S.root == NULLN) { S.root = leaf; S.tpar[leaf] = NULLN; return; }
        float llx = S.tlx[leaf], lly = S.tly[leaf], lhx = S.thx[leaf], lhy = S.thy[leaf];
        int index = S.root;
        for (int g = 0; !t_leaf(index); ++g) {
            if (g > LS::TN) { S.fault = MRP_FAULT_TREE_DOWN; break; }
            int c1 = S.tc1[index], c2 = S.tc2[index];
            float area = perim(S.tlx[index], S.tly[index], S.thx[index], S.thy[index]);
            float combinedArea = perim(fmin_(S.tlx[index], llx), fmin_(S.tly[index], lly), fmax_(S.thx[index], lhx), fmax_(S.thy[index], lhy));
            float cost = 2.0f * combinedArea;
            float inheritanceCost = 2.0f * (combinedArea - area);
            float cost1, cost2;
            {
                float na = perim(fmin_(llx, S.tlx[c1]), fmin_(lly, S.tly[c1]), fmax_(lhx, S.thx[c1]), fmax_(lhy, S.thy[c1]));
                if (t_leaf(c1)) cost1 = na + inheritanceCost;
                else { float oa = perim(S.tlx[c1], S.tly[c1], S.thx[c1], S.thy[c1]); cost1 = (na - oa) + inheritanceCost; }
            }
            {
                float na = perim(fmin_(llx, S.tlx[c2]), fmin_(lly, S.tly[c2]), fmax_(lhx, S.thx[c2]), fmax_(lhy, S.thy[c2]));
                if (t_leaf(c2)) cost2 = na + inheritanceCost;
                else { float oa = perim(S.tlx[c2], S.tly[c2], S.thx[c2], S.thy[c2]); cost2 = na - oa + inheritanceCost; }
            }
            if (cost < cost1 && cost < cost2) break;
            index = cost1 < cost2 ? c1 : c2;
        }
        int sibling = index;
        int oldParent = S.tpar[sibling];
        int np = t_alloc();
        S.tpar[np] = oldParent; S.tud[np] = -1;
        S.tlx[np] = fmin_(llx, S.tlx[sibling]); S.tly[np] = fmin_(lly, S.tly[sibling]);
        S.thx[np] = fmax_(lhx, S.thx[sibling]); S.thy[np] = fmax_(lhy, S.thy[sibling]);
        S.th[np] = S.th[sibling] + 1;
        if (oldParent != NULLN) { if (S.tc1[oldParent] == sibling) S.tc1[oldParent] = np; else S.tc2[oldParent] = np; }
        else S.root = np;
        S.tc1[np] = sibling; S.tc2[np] = leaf; S.tpar[sibling] = np; S.tpar[leaf] = np;
        t_fix_upwards(S.tpar[leaf]);
    }
    __device__ __forceinline__ void t_remove(int leaf) {
        if (leaf == S.root) { S.root = NULLN; return; }
        int parent = S.tpar[leaf];
        int grand = S.tpar[parent];
        int sibling = S.tc1[parent] == leaf ? S.tc2[parent] : S.tc1[parent];
        if (grand != NULLN) {
            if (S.tc1[grand] == parent) S.tc1[grand] = sibling; else S.tc2[grand] = sibling;
            S.tpar[sibling] = grand;
            t_free(parent);
            int index = grand;
            for (int g = 0; index != NULLN; ++g) {   // RemoveLeaf: Combine before height (same result as t_fix_upwards)
                if (g > LS::TN) { S.fault = MRP_FAULT_TREE_REMOVE; break; }
                index = t_balance(index);
                int c1 = S.tc1[index], c2 = S.tc2[index];
                t_combine_into(index, c1, c2);
                S.th[index] = 1 + max(S.th[c1], S.th[c2]);
                index = S.tpar[index];
            }
        } else {
            S.root = sibling; S.tpar[sibling] = NULLN; t_free(parent);
        }
    }
    __device__ __forceinline__ void buffer_move(int id) {
        if (S.moveCount >= LS::MOVE_N) { S.fault = MRP_FAULT_MOVE_BUFFER; return; }   // never in a valid world
        S.moveBuf[S.moveCount++] = id;
    }
    __device__ __forceinline__ void unbuffer_move(int id) { for (int i = 0; i < S.moveCount; ++i) if (S.moveBuf[i] == id) S.moveBuf[i] = NULLN; }

    // polygon AABB under a transform (b2PolygonShape::ComputeAABB)
    __device__ __forceinline__ void poly_aabb(const ShapeDef& s, Xf x, float& lx, float& ly, float& hx, float& hy) const {
        V2 lower = mul_xv(x, s.v[0]), upper = lower;
        for (int i = 1; i < s.count; ++i) { V2 v = mul_xv(x, s.v[i]); lower = vmin(lower, v); upper = vmax(upper, v); }
        lx = lower.x - s.radius; ly = lower.y - s.radius; hx = upper.x + s.radius; hy = upper.y + s.radius;
    }
    __device__ __forceinline__ void create_proxy(int f, Xf x) {
        float lx, ly, hx, hy;
        poly_aabb(L.shape[f], x, lx, ly, hx, hy);
        int id = t_alloc();
        S.tlx[id] = lx - AABB_EXT; S.tly[id] = ly - AABB_EXT; S.thx[id] = hx + AABB_EXT; S.thy[id] = hy + AABB_EXT;
        S.tud[id] = f; S.th[id] = 0;
        t_insert(id);
        S.proxy[f] = id;
        buffer_move(id);
    }
    __device__ __forceinline__ void destroy_proxy(int f) {
        int id = S.proxy[f];
        unbuffer_move(id);
        t_remove(id); t_free(id);
    }
    __device__ __forceinline__ void move_proxy(int id, float lx, float ly, float hx, float hy, V2 disp) {
        if (S.tlx[id] <= lx && S.tly[id] <= ly && hx <= S.thx[id] && hy <= S.thy[id]) return;   // Contains
        move_proxy_out(id, lx, ly, hx, hy, disp);
    }
    // b2DynamicTree::MoveProxy past its Contains test: reinsert the leaf with its new fat AABB
    __device__ __forceinline__ void move_proxy_out(int id, float lx, float ly, float hx, float hy, V2 disp) {
        t_remove(id);
        float blx = lx - AABB_EXT, bly = ly - AABB_EXT, bhx = hx + AABB_EXT, bhy = hy + AABB_EXT;
        V2 d = vmul(AABB_MUL, disp);
        if (d.x < 0.0f) blx += d.x; else bhx += d.x;
        if (d.y < 0.0f) bly += d.y; else bhy += d.y;
        S.tlx[id] = blx; S.tly[id] = bly; S.thx[id] = bhx; S.thy[id] = bhy;
        t_insert(id);
        buffer_move(id);
    }
    __device__ __forceinline__ bool fat_overlap(int a, int b) const {   // b2TestOverlap
        float d1x = S.tlx[b] - S.thx[a], d1y = S.tly[b] - S.thy[a];
        float d2x = S.tlx[a] - S.thx[b], d2y = S.tly[a] - S.thy[b];
        if (d1x > 0.0f || d1y > 0.0f) return false;
        if (d2x > 0.0f || d2y > 0.0f) return false;
        return true;
    }
    // b2Body::SynchronizeFixtures of every body flagged in `bflag` (b2World::Solve's end), on the whole
    // wave: lane f takes fixture f's swept AABB (its body's transform at the sweep start and now, the
    // float operations of sync_fixtures) and b2DynamicTree::MoveProxy's Contains test; a leaf's fat AABB
    // changes only in its own MoveProxy, so the test does not depend on the moves before it.  Thread 0
    // then reinserts the leaves that left their fat AABBs, in the reference's order (bodies from the
    // last created, fixtures newest first), which is the order the tree's shape depends on.
    __device__ __forceinline__ void sync_fixtures_coop(uint32_t bflag) {
        static_assert(NF <= 64, "one lane per fixture");
        const unsigned long long tf = MRP_NOW();
        const int f = tid < NF ? tid : 0;
        const int b = L.fix_body[f];
        const bool act = tid < NF && b < ND && ((bflag >> b) & 1u);
        bool out = false;
        if (act) {
            Xf x1; x1.q = rot(S.a0[b]);
            x1.p = vsub(v2(S.c0x[b], S.c0y[b]), mul_rv(x1.q, lc(b)));
            const Xf x2 = xf(b);
            float l1x, l1y, h1x, h1y, l2x, l2y, h2x, h2y;
            poly_aabb(L.shape[f], x1, l1x, l1y, h1x, h1y);
            poly_aabb(L.shape[f], x2, l2x, l2y, h2x, h2y);
            const V2 disp = vsub(x2.p, x1.p);
            const float lx = fmin_(l1x, l2x), ly = fmin_(l1y, l2y), hx = fmax_(h1x, h2x), hy = fmax_(h1y, h2y);
            const int id = S.proxy[f];
            out = !(S.tlx[id] <= lx && S.tly[id] <= ly && hx <= S.thx[id] && hy <= S.thy[id]);   // not Contains
            sh.u.fsync.lx[f] = lx; sh.u.fsync.ly[f] = ly; sh.u.fsync.hx[f] = hx; sh.u.fsync.hy[f] = hy;
            sh.u.fsync.dx[f] = disp.x; sh.u.fsync.dy[f] = disp.y;
        }
        const uint64_t moves = __builtin_amdgcn_ballot_w64(out);
        __syncthreads();
        if (tid == 0 && moves != 0ull) {
            for (int bb = ND - 1; bb >= 0; --bb) {
                if (!(bflag & (1u << bb))) continue;
                for (int k = L.body_nfix[bb] - 1; k >= 0; --k) {
                    const int ff = L.body_fix0[bb] + k;
                    if ((moves >> ff) & 1ull)
                        move_proxy_out(S.proxy[ff], sh.u.fsync.lx[ff], sh.u.fsync.ly[ff], sh.u.fsync.hx[ff], sh.u.fsync.hy[ff],
                                       v2(sh.u.fsync.dx[ff], sh.u.fsync.dy[ff]));
                }
            }
        }
        MRP_SUB(34, tf);
    }
    // b2Body::SynchronizeFixtures for a dynamic body, fixtures in fixture-list order (newest first)
    __device__ __forceinline__ void sync_fixtures(int b) {
        Xf x1; x1.q = rot_z(S.a0[b]);
        x1.p = vsub(v2(S.c0x[b], S.c0y[b]), mul_rv(x1.q, lc(b)));
        Xf x2 = xf(b);
        for (int k = L.body_nfix[b] - 1; k >= 0; --k) {
            int f = L.body_fix0[b] + k;
            float l1x, l1y, h1x, h1y, l2x, l2y, h2x, h2y;
            poly_aabb(L.shape[f], x1, l1x, l1y, h1x, h1y);
            poly_aabb(L.shape[f], x2, l2x, l2y, h2x, h2y);
            V2 disp = vsub(x2.p, x1.p);
            move_proxy(S.proxy[f], fmin_(l1x, l2x), fmin_(l1y, l2y), fmax_(h1x, h2x), fmax_(h1y, h2y), disp);
        }
    }

    // ------------------------------------------------------------------ contacts
    __device__ __forceinline__ void contact_event(int c, int value) {   // ContactDetector (multi_robot_puzzle_00.py:92-111)
        // v3's detector (core.py:46-61) compares Robot wrappers with b2Body objects: never a match
        if (D::V == 3) return;
        int bA = L.fix_body[S.cfa[c]], bB = L.fix_body[S.cfb[c]];
        for (int i = 0; i < NA; ++i) {
            int ag = NB + i;
            if (ag == bA || ag == bB) {
                if (bA == 0 || bB == 0) S.goal_contact[i] = value;
                if (bA >= ND || bB >= ND) S.wall_contact = value;
            }
        }
    }
    __device__ __forceinline__ void add_pair(int fa, int fb) {   // b2ContactManager::AddPair
        int bA = L.fix_body[fa], bB = L.fix_body[fb];
        if (bA == bB) return;
        for (int c = S.cHead, g_ = 0; c != NULLN && list_ok(g_); c = S.cnext[c]) {
            if ((S.cfa[c] == fa && S.cfb[c] == fb) || (S.cfa[c] == fb && S.cfb[c] == fa)) return;
        }
        if (!is_dyn(bA) && !is_dyn(bB)) return;
        int c = S.cFree;
        if ((unsigned)c >= (unsigned)C) { S.fault = MRP_FAULT_CONTACT_POOL; return; }   // never in a valid world
        S.cFree = S.cnext[c];
        if (c >= S.cHW) S.cHW = c + 1;
        S.cfa[c] = fa; S.cfb[c] = fb; S.cflags[c] = CF_ENABLED; S.ctoiCount[c] = 0; S.ctoi[c] = 1.0f;
        S.cfric[c] = sqrtf(L.fix_friction[fa] * L.fix_friction[fb]);
        S.mpc[c] = 0;
        S.cprev[c] = NULLN; S.cnext[c] = S.cHead;
        if (S.cHead != NULLN) S.cprev[S.cHead] = c;
        S.cHead = c;
        ++S.cCount;
    }
    __device__ __forceinline__ void destroy_contact(int c, bool events) {   // b2ContactManager::Destroy
        if (events && (S.cflags[c] & CF_TOUCHING)) contact_event(c, 0);
        int p = S.cprev[c], n = S.cnext[c];
        if (p != NULLN) S.cnext[p] = n;
        if (n != NULLN) S.cprev[n] = p;
        if (S.cHead == c) S.cHead = n;
        S.cnext[c] = S.cFree; S.cFree = c;
        --S.cCount;
    }
    // b2BroadPhase::UpdatePairs + AddPair: pairs (lower proxy id, higher id) with at least one
    // moved proxy and overlapping fat AABBs, visited in sorted order == Box2D's sorted pair buffer.
    // Cooperative: every thread of the wave calls it; the O(P^2) overlap tests run in parallel,
    // the order-sensitive AddPair calls run on thread 0 in sorted order.
    __device__ __forceinline__ void find_new_contacts_coop() {
        if (tid == 0) {
            typename LS::PMask moved = 0;
            for (int i = 0; i < S.moveCount; ++i) if (S.moveBuf[i] != NULLN) moved |= (typename LS::PMask)1 << S.moveBuf[i];
            S.moveCount = 0;
            int n = 0;
            if (moved)
                for (int a = 0; a < LS::TN; ++a) if (S.tud[a] >= 0 && t_leaf(a)) sh.prox[n++] = a;
            sh.nprox = n;
            sh.moved = moved;
        }
        __syncthreads();
        const int n = sh.nprox;
        const typename LS::PMask moved = sh.moved;
        const int npairs = n * (n - 1) / 2;
        for (int p = tid; p < npairs; p += 64) {
            int i = 0, q = p;
            while (q >= n - 1 - i) {
                if (i >= n - 1) { S.fault = MRP_FAULT_PAIR_DECODE; i = 0; q = 0; break; }
                q -= n - 1 - i; ++i;
            }
            int a = sh.prox[i], b = sh.prox[i + 1 + q];
            sh.u.pover[p] = ((((moved >> a) | (moved >> b)) & 1u) && fat_overlap(a, b)) ? 1 : 0;
        }
        __syncthreads();
        if (tid == 0) {
            int p = 0;
            for (int i = 0; i < n; ++i)
                for (int j = i + 1; j < n; ++j, ++p)
                    if (sh.u.pover[p]) add_pair(S.tud[sh.prox[i]], S.tud[sh.prox[j]]);
        }
        __syncthreads();
    }

    // ---------------------------------------------------------------- narrow phase (b2CollidePolygons)
    __device__ __forceinline__ static uint32_t cf_make(int iA, int iB, int tA, int tB) {
        return (uint32_t)(uint8_t)iA | ((uint32_t)(uint8_t)iB << 8) | ((uint32_t)(uint8_t)tA << 16) | ((uint32_t)(uint8_t)tB << 24);
    }
    __device__ __forceinline__ static float find_max_separation(int& edge, const ShapeDef& p1, Xf x1, const ShapeDef& p2, Xf x2) {
        Xf x = mulT_xx(x2, x1);
        int best = 0; float maxSep = -FLT_MAXV;
        for (int i = 0; i < p1.count; ++i) {
            V2 n = mul_rv(x.q, p1.n[i]);
            V2 v1 = mul_xv(x, p1.v[i]);
            float si = FLT_MAXV;
            for (int j = 0; j < p2.count; ++j) { float sij = vdot(n, vsub(p2.v[j], v1)); if (sij < si) si = sij; }
            if (si > maxSep) { maxSep = si; best = i; }
        }
        edge = best;
        return maxSep;
    }
    // find_max_separation over a group of G lanes (G a power of two <= 8; the group's lanes are
    // consecutive and `sub` is this lane's place in it): lane sub scans edges sub, sub + G, ... in
    // the reference's order and rule (strict >, so the first index of the maximum wins), then the
    // group reduces to the larger separation, the smaller edge among equals.  An edge that never
    // beats the reference's running maximum (NaN, or not above -FLT_MAX) takes no part; with none
    // left the result is the reference's (edge 0, -FLT_MAX).  Same bits as find_max_separation.
    __device__ __forceinline__ static float find_max_separation_grp(int& edge, const ShapeDef& p1, Xf x1, const ShapeDef& p2, Xf x2,
                                                                    int sub, int G) {
        Xf x = mulT_xx(x2, x1);
        int best = MAX_POLY; float maxSep = -FLT_MAXV;
        for (int i = sub; i < p1.count; i += G) {
            V2 n = mul_rv(x.q, p1.n[i]);
            V2 v1 = mul_xv(x, p1.v[i]);
            float si = FLT_MAXV;
            for (int j = 0; j < p2.count; ++j) { float sij = vdot(n, vsub(p2.v[j], v1)); if (sij < si) si = sij; }
            if (si > maxSep) { maxSep = si; best = i; }
        }
        for (int m = 1; m < G; m <<= 1) {
            const float os = __shfl_xor(maxSep, m, G);
            const int ob = __shfl_xor(best, m, G);
            if (ob < MAX_POLY && (best == MAX_POLY || os > maxSep || (os == maxSep && ob < best))) { maxSep = os; best = ob; }
        }
        edge = best == MAX_POLY ? 0 : best;
        return best == MAX_POLY ? -FLT_MAXV : maxSep;
    }
    // b2ClipSegmentToLine with the two in/out vertices kept in registers
    __device__ __forceinline__ static int clip(ClipV& o0, ClipV& o1, const ClipV& i0, const ClipV& i1, V2 normal, float offset, int vertexIndexA) {
        int numOut = 0;
        float d0 = vdot(normal, i0.v) - offset;
        float d1 = vdot(normal, i1.v) - offset;
        if (d0 <= 0.0f) { o0 = i0; numOut = 1; }
        if (d1 <= 0.0f) { if (numOut == 0) o0 = i1; else o1 = i1; ++numOut; }
        if (d0 * d1 < 0.0f) {   // exactly one endpoint was kept, so this fills slot 1
            float interp = d0 / (d0 - d1);
            o1.v = vadd(i0.v, vmul(interp, vsub(i1.v, i0.v)));
            o1.id = cf_make(vertexIndexA, (int)((i0.id >> 8) & 0xff), 0, 1);
            ++numOut;
        }
        return numOut;
    }
    // manifold scratch: parallel slot k (narrow phase) or the serial slot (k < 0)
    __device__ __forceinline__ int& m_pc(int k) { return k < 0 ? sh.spc : sh.u.col.tpc[k]; }
    __device__ __forceinline__ int& m_type(int k) { return k < 0 ? sh.stype : sh.u.col.ttype[k]; }
    __device__ __forceinline__ float& m_lnx(int k) { return k < 0 ? sh.slnx : sh.u.col.tlnx[k]; }
    __device__ __forceinline__ float& m_lny(int k) { return k < 0 ? sh.slny : sh.u.col.tlny[k]; }
    __device__ __forceinline__ float& m_lpx(int k) { return k < 0 ? sh.slpx : sh.u.col.tlpx[k]; }
    __device__ __forceinline__ float& m_lpy(int k) { return k < 0 ? sh.slpy : sh.u.col.tlpy[k]; }
    __device__ __forceinline__ float& m_px(int i, int k) { return k < 0 ? sh.spx[i] : sh.u.col.tpx[i][k]; }
    __device__ __forceinline__ float& m_py(int i, int k) { return k < 0 ? sh.spy[i] : sh.u.col.tpy[i][k]; }
    __device__ __forceinline__ uint32_t& m_id(int i, int k) { return k < 0 ? sh.smid[i] : sh.u.col.tmid[i][k]; }
    // b2CollidePolygons into manifold scratch slot k; with G > 1 the G lanes of a group run it
    // together (find_max_separation_grp), every lane computing the same values for the rest
    __device__ __forceinline__ void collide_polygons(int k, const ShapeDef& pA, Xf xA, const ShapeDef& pB, Xf xB, int sub = 0, int G = 1) {
        m_pc(k) = 0;
        float totalRadius = pA.radius + pB.radius;
        int edgeA = 0;
        float sepA = G > 1 ? find_max_separation_grp(edgeA, pA, xA, pB, xB, sub, G) : find_max_separation(edgeA, pA, xA, pB, xB);
        if (sepA > totalRadius) return;
        int edgeB = 0;
        float sepB = G > 1 ? find_max_separation_grp(edgeB, pB, xB, pA, xA, sub, G) : find_max_separation(edgeB, pB, xB, pA, xA);
        if (sepB > totalRadius) return;
        const float k_tol = 0.1f * LINEAR_SLOP;
        bool flip = sepB > sepA + k_tol;
        const ShapeDef& p1 = flip ? pB : pA;
        const ShapeDef& p2 = flip ? pA : pB;
        Xf x1 = flip ? xB : xA, x2 = flip ? xA : xB;
        int edge1 = flip ? edgeB : edgeA;
        m_type(k) = flip ? MT_FACEB : MT_FACEA;
        ClipV inc0, inc1;   // incident edge
        {
            V2 normal1 = mulT_rv(x2.q, mul_rv(x1.q, p1.n[edge1]));
            int index = 0; float minDot = FLT_MAXV;
            for (int i = 0; i < p2.count; ++i) { float d = vdot(normal1, p2.n[i]); if (d < minDot) { minDot = d; index = i; } }
            int i1 = index, i2 = i1 + 1 < p2.count ? i1 + 1 : 0;
            inc0.v = mul_xv(x2, p2.v[i1]); inc0.id = cf_make(edge1, i1, 1, 0);
            inc1.v = mul_xv(x2, p2.v[i2]); inc1.id = cf_make(edge1, i2, 1, 0);
        }
        int iv1 = edge1, iv2 = edge1 + 1 < p1.count ? edge1 + 1 : 0;
        V2 v11 = p1.v[iv1], v12 = p1.v[iv2];
        V2 localTangent = vsub(v12, v11);
        vnormalize(localTangent);
        V2 localNormal = vcross_vs(localTangent, 1.0f);
        V2 planePoint = vmul(0.5f, vadd(v11, v12));
        V2 tangent = mul_rv(x1.q, localTangent);
        V2 normal = vcross_vs(tangent, 1.0f);
        v11 = mul_xv(x1, v11); v12 = mul_xv(x1, v12);
        float frontOffset = vdot(normal, v11);
        float side1 = -vdot(tangent, v11) + totalRadius;
        float side2 = vdot(tangent, v12) + totalRadius;
        ClipV a0, a1, b0, b1;
        if (clip(a0, a1, inc0, inc1, vneg(tangent), side1, iv1) < 2) return;
        if (clip(b0, b1, a0, a1, tangent, side2, iv2) < 2) return;
        m_lnx(k) = localNormal.x; m_lny(k) = localNormal.y;
        m_lpx(k) = planePoint.x; m_lpy(k) = planePoint.y;
        int pc = 0;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const ClipV& cv = i == 0 ? b0 : b1;
            float sep = vdot(normal, cv.v) - frontOffset;
            if (sep <= totalRadius) {
                V2 lp = mulT_xv(x2, cv.v);
                uint32_t id = cv.id;
                if (flip) {
                    uint32_t q0 = id & 0xff, q1 = (id >> 8) & 0xff, ta = (id >> 16) & 0xff, tb = (id >> 24) & 0xff;
                    id = q1 | (q0 << 8) | (tb << 16) | (ta << 24);
                }
                if (pc == 0) { m_px(0, k) = lp.x; m_py(0, k) = lp.y; m_id(0, k) = id; }
                else { m_px(1, k) = lp.x; m_py(1, k) = lp.y; m_id(1, k) = id; }
                ++pc;
            }
        }
        m_pc(k) = pc;
    }
    // second half of b2Contact::Update: adopt manifold scratch slot k, match feature ids to
    // carry the warm-start impulses, update the touching flag, fire Begin/End events
    __device__ __forceinline__ void contact_commit(int c, int k) {
        int oldCount = S.mpc[c];
        uint32_t oid0 = S.mid[0][c], oid1 = S.mid[1][c];
        float on0 = S.mni[0][c], on1 = S.mni[1][c], ot0 = S.mti[0][c], ot1 = S.mti[1][c];
        S.cflags[c] |= CF_ENABLED;
        bool wasTouching = (S.cflags[c] & CF_TOUCHING) != 0;
        int pcount = m_pc(k);
        S.mpc[c] = pcount;
        if (pcount > 0) {
            S.mtype[c] = m_type(k);
            S.mlnx[c] = m_lnx(k); S.mlny[c] = m_lny(k); S.mlpx[c] = m_lpx(k); S.mlpy[c] = m_lpy(k);
        }
        for (int i = 0; i < pcount; ++i) {
            uint32_t id2 = m_id(i, k);
            S.mpx[i][c] = m_px(i, k); S.mpy[i][c] = m_py(i, k); S.mid[i][c] = id2;
            float ni = 0.0f, ti = 0.0f;
            if (oldCount > 0 && oid0 == id2) { ni = on0; ti = ot0; }
            else if (oldCount > 1 && oid1 == id2) { ni = on1; ti = ot1; }
            S.mni[i][c] = ni; S.mti[i][c] = ti;
        }
        bool touching = pcount > 0;
        if (touching) S.cflags[c] |= CF_TOUCHING; else S.cflags[c] &= ~CF_TOUCHING;
        if (!wasTouching && touching) contact_event(c, 1);
        if (wasTouching && !touching) contact_event(c, 0);
    }
    // b2Contact::Update on one contact (serial callers: TOI)
    __device__ __forceinline__ void contact_update(int c) {
        int fa = S.cfa[c], fb = S.cfb[c];
        collide_polygons(-1, L.shape[fa], xf(L.fix_body[fa]), L.shape[fb], xf(L.fix_body[fb]));
        contact_commit(c, -1);
    }
    // b2ContactManager::Collide.  Cooperative: thread 0 snapshots the contact list, all threads
    // run the broad-phase overlap test + SAT narrow phase of one contact each, then thread 0
    // destroys / commits in list order (events fire in the reference's order).
    __device__ __forceinline__ void collide_coop() {
        const unsigned long long tc0 = MRP_NOW();
        if (tid == 0) {
            int n = 0;
            for (int c = S.cHead, g_ = 0; c != NULLN && list_ok(g_); c = S.cnext[c]) sh.clist[n++] = c;
            sh.ccount = n;
        }
        __syncthreads();
        const int n = sh.ccount;
        // up to 32 contacts: a group of G = 8, 4 or 2 lanes per contact shares its SAT edge scans
        // (collide_polygons with G > 1); more: one lane per contact
        const int G = n <= 8 ? 8 : (n <= 16 ? 4 : (n <= 32 ? 2 : 1));
        if (G > 1) {
            const int g = tid / G, sub = tid & (G - 1);
            if (g < n) {
                int c = sh.clist[g];
                int fa = S.cfa[c], fb = S.cfb[c];
                bool ov = fat_overlap(S.proxy[fa], S.proxy[fb]);
                if (sub == 0) sh.cover[g] = ov ? 1 : 0;
                if (ov) collide_polygons(g, L.shape[fa], xf(L.fix_body[fa]), L.shape[fb], xf(L.fix_body[fb]), sub, G);
            }
        } else {
            for (int i = tid; i < n; i += 64) {
                int c = sh.clist[i];
                int fa = S.cfa[c], fb = S.cfb[c];
                bool ov = fat_overlap(S.proxy[fa], S.proxy[fb]);
                sh.cover[i] = ov ? 1 : 0;
                if (ov) collide_polygons(i, L.shape[fa], xf(L.fix_body[fa]), L.shape[fb], xf(L.fix_body[fb]));
            }
        }
        // touching contacts after this update decide how much solver work the lane has left: the
        // contact-heavy lanes set the kernel's duration, so they take issue priority from here on
        int touching = 0;
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + tid;
            const bool t = i < n && sh.cover[i] && sh.u.col.tpc[i] > 0;
            touching += __popcll(__ballot(t));
        }
        touching = __builtin_amdgcn_readfirstlane(touching);
        if (tid == 0) S.touching += touching;
        step_prio = touching >= 4 ? 2 : (touching >= 2 ? 1 : 0);
        if (prio_floor > step_prio) step_prio = prio_floor;
        set_prio(step_prio);
        __syncthreads();
#ifndef MRP_STAMPS_TOI
        MRP_SUB(22, tc0);   // collide split: contact-list snapshot + narrow phase of every contact
#endif
        const unsigned long long tc1 = MRP_NOW();
        if (tid == 0) {
            for (int i = 0; i < n; ++i) {
                int c = sh.clist[i];
                if (!sh.cover[i]) destroy_contact(c, true);
                else contact_commit(c, i);
            }
        }
        __syncthreads();
#ifndef MRP_STAMPS_TOI
        MRP_SUB(23, tc1);   // collide split: serial commit (feature-id matching, events, destroys)
#endif
    }

    // wave issue priority (s_setprio takes an immediate); `level` must be wave-uniform
    __device__ __forceinline__ static void set_prio(int level) {
        level = __builtin_amdgcn_readfirstlane(level);
        if (level >= 3) __builtin_amdgcn_s_setprio(3);
        else if (level == 2) __builtin_amdgcn_s_setprio(2);
        else if (level == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    }

    // ---------------------------------------------------------------- contact solver
    __device__ __forceinline__ float body_invMass(int b) const { return L.invMass[b]; }
    __device__ __forceinline__ float body_invI(int b) const { return L.invI[b]; }

    __device__ __forceinline__ void solver_init(Isl& is, VC* vcs, PC* pcs, bool warm, float dtRatio) {
        for (int i = 0; i < is.nc; ++i) {
            int c = is.contacts[i];
            int fa = S.cfa[c], fb = S.cfb[c];
            int bA = L.fix_body[fa], bB = L.fix_body[fb];
            int pcount = S.mpc[c];
            VC& vc = vcs[i];
            vc.friction = S.cfric[c];
            vc.iaI = is.index[bA]; vc.ibI = is.index[bB];
            vc.mA = L.invMass[bA]; vc.mB = L.invMass[bB]; vc.iA = L.invI[bA]; vc.iB = L.invI[bB];
            vc.slot = c; vc.pointCount = pcount;
            vc.k0 = vc.k1 = vc.k3 = 0.0f; vc.nm0 = vc.nm1 = vc.nm3 = 0.0f;
            PC& pc = pcs[i];
            pc.lcAx = L.lcx[bA]; pc.lcAy = L.lcy[bA]; pc.lcBx = L.lcx[bB]; pc.lcBy = L.lcy[bB];
            pc.lnx = S.mlnx[c]; pc.lny = S.mlny[c]; pc.lpx0 = S.mlpx[c]; pc.lpy0 = S.mlpy[c];
            pc.pointCount = pcount; pc.rA = L.shape[fa].radius; pc.rB = L.shape[fb].radius; pc.type = S.mtype[c];
            for (int j = 0; j < pcount; ++j) {
                if (warm) { vc.ni[j] = dtRatio * S.mni[j][c]; vc.ti[j] = dtRatio * S.mti[j][c]; }
                else { vc.ni[j] = 0.0f; vc.ti[j] = 0.0f; }
                vc.rAx[j] = vc.rAy[j] = vc.rBx[j] = vc.rBy[j] = 0.0f;
                vc.nmass[j] = 0.0f; vc.tmass[j] = 0.0f; vc.vbias[j] = 0.0f;
                pc.lpx[j] = S.mpx[j][c]; pc.lpy[j] = S.mpy[j][c];
            }
        }
    }
    __device__ __forceinline__ void solver_init_velocity(Isl& is, VC* vcs, PC* pcs) {
        for (int i = 0; i < is.nc; ++i) {
            VC& vc = vcs[i]; PC& pc = pcs[i];
            int c = vc.slot;
            const float restitution = fmax_(L.fix_restitution[S.cfa[c]], L.fix_restitution[S.cfb[c]]);
            int ia = vc.iaI, ib = vc.ibI;
            float mA = vc.mA, mB = vc.mB, iA = vc.iA, iB = vc.iB;
            V2 cA = v2(is.pcx[ia], is.pcy[ia]); float aA = is.pa[ia];
            V2 vA = v2(is.vvx[ia], is.vvy[ia]); float wA = is.vw[ia];
            V2 cB = v2(is.pcx[ib], is.pcy[ib]); float aB = is.pa[ib];
            V2 vB = v2(is.vvx[ib], is.vvy[ib]); float wB = is.vw[ib];
            Xf xA, xB;
            xA.q = rot_z(aA); xB.q = rot_z(aB);
            xA.p = vsub(cA, mul_rv(xA.q, v2(pc.lcAx, pc.lcAy)));
            xB.p = vsub(cB, mul_rv(xB.q, v2(pc.lcBx, pc.lcBy)));
            // b2WorldManifold::Initialize
            V2 normal; V2 pts[2];
            int mpcount = S.mpc[c];
            if (S.mtype[c] == MT_FACEA) {
                normal = mul_rv(xA.q, v2(S.mlnx[c], S.mlny[c]));
                V2 planePoint = mul_xv(xA, v2(S.mlpx[c], S.mlpy[c]));
#pragma unroll
                for (int j = 0; j < 2; ++j) {   // constant indices: pts stays in registers (no scratch)
                    if (j >= mpcount) break;
                    V2 clipPoint = mul_xv(xB, v2(S.mpx[j][c], S.mpy[j][c]));
                    V2 pA = vadd(clipPoint, vmul(pc.rA - vdot(vsub(clipPoint, planePoint), normal), normal));
                    V2 pB = vsub(clipPoint, vmul(pc.rB, normal));
                    pts[j] = vmul(0.5f, vadd(pA, pB));
                }
            } else {
                normal = mul_rv(xB.q, v2(S.mlnx[c], S.mlny[c]));
                V2 planePoint = mul_xv(xB, v2(S.mlpx[c], S.mlpy[c]));
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (j >= mpcount) break;
                    V2 clipPoint = mul_xv(xA, v2(S.mpx[j][c], S.mpy[j][c]));
                    V2 pB = vadd(clipPoint, vmul(pc.rB - vdot(vsub(clipPoint, planePoint), normal), normal));
                    V2 pA = vsub(clipPoint, vmul(pc.rA, normal));
                    pts[j] = vmul(0.5f, vadd(pA, pB));
                }
                normal = vneg(normal);
            }
            vc.nx = normal.x; vc.ny = normal.y;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (j >= vc.pointCount) break;
                V2 rA = vsub(pts[j], cA), rB = vsub(pts[j], cB);
                vc.rAx[j] = rA.x; vc.rAy[j] = rA.y; vc.rBx[j] = rB.x; vc.rBy[j] = rB.y;
                float rnA = vcross(rA, normal), rnB = vcross(rB, normal);
                float kNormal = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
                vc.nmass[j] = kNormal > 0.0f ? 1.0f / kNormal : 0.0f;
                V2 tangent = vcross_vs(normal, 1.0f);
                float rtA = vcross(rA, tangent), rtB = vcross(rB, tangent);
                float kTangent = mA + mB + iA * rtA * rtA + iB * rtB * rtB;
                vc.tmass[j] = kTangent > 0.0f ? 1.0f / kTangent : 0.0f;
                vc.vbias[j] = 0.0f;
                V2 dvr = vsub(vsub(vadd(vB, vcross_sv(wB, rB)), vA), vcross_sv(wA, rA));
                float vRel = vdot(normal, dvr);
                if (vRel < -VELOCITY_THRESHOLD) vc.vbias[j] = -restitution * vRel;
            }
            if (vc.pointCount == 2) {
                float rn1A = vcross(v2(vc.rAx[0], vc.rAy[0]), normal), rn1B = vcross(v2(vc.rBx[0], vc.rBy[0]), normal);
                float rn2A = vcross(v2(vc.rAx[1], vc.rAy[1]), normal), rn2B = vcross(v2(vc.rBx[1], vc.rBy[1]), normal);
                float k11 = mA + mB + iA * rn1A * rn1A + iB * rn1B * rn1B;
                float k22 = mA + mB + iA * rn2A * rn2A + iB * rn2B * rn2B;
                float k12 = mA + mB + iA * rn1A * rn2A + iB * rn1B * rn2B;
                const float k_maxConditionNumber = 1000.0f;
                if (k11 * k11 < k_maxConditionNumber * (k11 * k22 - k12 * k12)) {
                    vc.k0 = k11; vc.k1 = k12; vc.k3 = k22;   // k2 = k12 too
                    float a = vc.k0, b = vc.k1, cc = vc.k1, d = vc.k3;
                    float det = a * d - b * cc;
                    if (det != 0.0f) det = 1.0f / det;
                    vc.nm0 = det * d; vc.nm1 = -det * cc; vc.nm3 = det * a;   // nm2 = -det * b == nm1
                } else {
                    vc.pointCount = 1;
                }
            }
        }
    }
    __device__ __forceinline__ void solver_warm_start(Isl& is, VC* vcs) {
        for (int i = 0; i < is.nc; ++i) {
            VC& vc = vcs[i];
            int ia = vc.iaI, ib = vc.ibI;
            V2 vA = v2(is.vvx[ia], is.vvy[ia]); float wA = is.vw[ia];
            V2 vB = v2(is.vvx[ib], is.vvy[ib]); float wB = is.vw[ib];
            V2 normal = v2(vc.nx, vc.ny), tangent = vcross_vs(normal, 1.0f);
            for (int j = 0; j < vc.pointCount; ++j) {
                V2 P = vadd(vmul(vc.ni[j], normal), vmul(vc.ti[j], tangent));
                wA -= vc.iA * vcross(v2(vc.rAx[j], vc.rAy[j]), P);
                vA = vsub(vA, vmul(vc.mA, P));
                wB += vc.iB * vcross(v2(vc.rBx[j], vc.rBy[j]), P);
                vB = vadd(vB, vmul(vc.mB, P));
            }
            is.vvx[ia] = vA.x; is.vvy[ia] = vA.y; is.vw[ia] = wA;
            is.vvx[ib] = vB.x; is.vvy[ib] = vB.y; is.vw[ib] = wB;
        }
    }
    __device__ __forceinline__ void solver_velocity(Isl& is, VC* vcs) {   // b2ContactSolver::SolveVelocityConstraints
        for (int i = 0; i < is.nc; ++i) {
            VC& vc = vcs[i];
            int ia = vc.iaI, ib = vc.ibI;
            float mA = vc.mA, iA = vc.iA, mB = vc.mB, iB = vc.iB;
            V2 vA = v2(is.vvx[ia], is.vvy[ia]); float wA = is.vw[ia];
            V2 vB = v2(is.vvx[ib], is.vvy[ib]); float wB = is.vw[ib];
            V2 normal = v2(vc.nx, vc.ny), tangent = vcross_vs(normal, 1.0f);
            float friction = vc.friction;
            for (int j = 0; j < vc.pointCount; ++j) {
                V2 rA = v2(vc.rAx[j], vc.rAy[j]), rB = v2(vc.rBx[j], vc.rBy[j]);
                V2 dv = vsub(vsub(vadd(vB, vcross_sv(wB, rB)), vA), vcross_sv(wA, rA));
                float vt = vdot(dv, tangent) - 0.0f;
                float lambda = vc.tmass[j] * (-vt);
                float maxFriction = friction * vc.ni[j];
                float newImpulse = fclamp(vc.ti[j] + lambda, -maxFriction, maxFriction);
                lambda = newImpulse - vc.ti[j];
                vc.ti[j] = newImpulse;
                V2 P = vmul(lambda, tangent);
                vA = vsub(vA, vmul(mA, P));
                wA -= iA * vcross(rA, P);
                vB = vadd(vB, vmul(mB, P));
                wB += iB * vcross(rB, P);
            }
            if (vc.pointCount == 1) {
                V2 rA = v2(vc.rAx[0], vc.rAy[0]), rB = v2(vc.rBx[0], vc.rBy[0]);
                V2 dv = vsub(vsub(vadd(vB, vcross_sv(wB, rB)), vA), vcross_sv(wA, rA));
                float vn = vdot(dv, normal);
                float lambda = -vc.nmass[0] * (vn - vc.vbias[0]);
                float newImpulse = fmax_(vc.ni[0] + lambda, 0.0f);
                lambda = newImpulse - vc.ni[0];
                vc.ni[0] = newImpulse;
                V2 P = vmul(lambda, normal);
                vA = vsub(vA, vmul(mA, P));
                wA -= iA * vcross(rA, P);
                vB = vadd(vB, vmul(mB, P));
                wB += iB * vcross(rB, P);
            } else {
                V2 r1A = v2(vc.rAx[0], vc.rAy[0]), r1B = v2(vc.rBx[0], vc.rBy[0]);
                V2 r2A = v2(vc.rAx[1], vc.rAy[1]), r2B = v2(vc.rBx[1], vc.rBy[1]);
                V2 a = v2(vc.ni[0], vc.ni[1]);
                V2 dv1 = vsub(vsub(vadd(vB, vcross_sv(wB, r1B)), vA), vcross_sv(wA, r1A));
                V2 dv2 = vsub(vsub(vadd(vB, vcross_sv(wB, r2B)), vA), vcross_sv(wA, r2A));
                float vn1 = vdot(dv1, normal), vn2 = vdot(dv2, normal);
                V2 b = v2(vn1 - vc.vbias[0], vn2 - vc.vbias[1]);
                b = vsub(b, v2(vc.k0 * a.x + vc.k1 * a.y, vc.k1 * a.x + vc.k3 * a.y));
                V2 x;
                bool ok = false;
                x = vneg(v2(vc.nm0 * b.x + vc.nm1 * b.y, vc.nm1 * b.x + vc.nm3 * b.y));
                if (x.x >= 0.0f && x.y >= 0.0f) ok = true;
                if (!ok) {
                    x.x = -vc.nmass[0] * b.x; x.y = 0.0f;
                    vn2 = vc.k1 * x.x + b.y;
                    if (x.x >= 0.0f && vn2 >= 0.0f) ok = true;
                }
                if (!ok) {
                    x.x = 0.0f; x.y = -vc.nmass[1] * b.y;
                    vn1 = vc.k1 * x.y + b.x;
                    if (x.y >= 0.0f && vn1 >= 0.0f) ok = true;
                }
                if (!ok) {
                    x.x = 0.0f; x.y = 0.0f; vn1 = b.x; vn2 = b.y;
                    if (vn1 >= 0.0f && vn2 >= 0.0f) ok = true;
                }
                if (ok) {
                    V2 d = vsub(x, a);
                    V2 P1 = vmul(d.x, normal), P2 = vmul(d.y, normal);
                    vA = vsub(vA, vmul(mA, vadd(P1, P2)));
                    wA -= iA * (vcross(r1A, P1) + vcross(r2A, P2));
                    vB = vadd(vB, vmul(mB, vadd(P1, P2)));
                    wB += iB * (vcross(r1B, P1) + vcross(r2B, P2));
                    vc.ni[0] = x.x; vc.ni[1] = x.y;
                }
            }
            is.vvx[ia] = vA.x; is.vvy[ia] = vA.y; is.vw[ia] = wA;
            is.vvx[ib] = vB.x; is.vvy[ib] = vB.y; is.vw[ib] = wB;
        }
    }
    __device__ __forceinline__ void solver_store(Isl& is, VC* vcs) {
        for (int i = 0; i < is.nc; ++i) {
            VC& vc = vcs[i];
            for (int j = 0; j < vc.pointCount; ++j) { S.mni[j][vc.slot] = vc.ni[j]; S.mti[j][vc.slot] = vc.ti[j]; }
        }
    }
    __device__ __forceinline__ bool solver_position(Isl& is, const VC* vcs, PC* pcs, bool toi, int toiA, int toiB) {
        float minSep = 0.0f;
        for (int i = 0; i < is.nc; ++i) {
            PC& pc = pcs[i];
            const VC& vc = vcs[i];
            int ia = vc.iaI, ib = vc.ibI;
            float mA, iA, mB, iB;
            if (!toi) { mA = vc.mA; iA = vc.iA; mB = vc.mB; iB = vc.iB; }
            else {
                mA = 0.0f; iA = 0.0f; if (ia == toiA || ia == toiB) { mA = vc.mA; iA = vc.iA; }
                mB = 0.0f; iB = 0.0f; if (ib == toiA || ib == toiB) { mB = vc.mB; iB = vc.iB; }
            }
            V2 cA = v2(is.pcx[ia], is.pcy[ia]); float aA = is.pa[ia];
            V2 cB = v2(is.pcx[ib], is.pcy[ib]); float aB = is.pa[ib];
            for (int j = 0; j < pc.pointCount; ++j) {
                Xf xA, xB;
                xA.q = rot_z(aA); xB.q = rot_z(aB);
                xA.p = vsub(cA, mul_rv(xA.q, v2(pc.lcAx, pc.lcAy)));
                xB.p = vsub(cB, mul_rv(xB.q, v2(pc.lcBx, pc.lcBy)));
                V2 normal, point; float sep;
                if (pc.type == MT_FACEA) {
                    normal = mul_rv(xA.q, v2(pc.lnx, pc.lny));
                    V2 planePoint = mul_xv(xA, v2(pc.lpx0, pc.lpy0));
                    V2 clipPoint = mul_xv(xB, v2(pc.lpx[j], pc.lpy[j]));
                    sep = vdot(vsub(clipPoint, planePoint), normal) - pc.rA - pc.rB;
                    point = clipPoint;
                } else {
                    normal = mul_rv(xB.q, v2(pc.lnx, pc.lny));
                    V2 planePoint = mul_xv(xB, v2(pc.lpx0, pc.lpy0));
                    V2 clipPoint = mul_xv(xA, v2(pc.lpx[j], pc.lpy[j]));
                    sep = vdot(vsub(clipPoint, planePoint), normal) - pc.rA - pc.rB;
                    point = clipPoint;
                    normal = vneg(normal);
                }
                V2 rA = vsub(point, cA), rB = vsub(point, cB);
                minSep = fmin_(minSep, sep);
                float Cc = fclamp((toi ? TOI_BAUMGARTE : BAUMGARTE) * (sep + LINEAR_SLOP), -MAX_LINEAR_CORRECTION, 0.0f);
                float rnA = vcross(rA, normal), rnB = vcross(rB, normal);
                float K = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
                float impulse = K > 0.0f ? -Cc / K : 0.0f;
                V2 Pv = vmul(impulse, normal);
                cA = vsub(cA, vmul(mA, Pv));
                aA -= iA * vcross(rA, Pv);
                cB = vadd(cB, vmul(mB, Pv));
                aB += iB * vcross(rB, Pv);
            }
            is.pcx[ia] = cA.x; is.pcy[ia] = cA.y; is.pa[ia] = aA;
            is.pcx[ib] = cB.x; is.pcy[ib] = cB.y; is.pa[ib] = aB;
        }
        return toi ? (minSep >= -1.5f * LINEAR_SLOP) : (minSep >= -3.0f * LINEAR_SLOP);
    }
    // ---------------------------------------------------------------- lane-distributed velocity sweeps
    // b2ContactSolver::SolveVelocityConstraints x `iters` with the island's constraint data held
    // in VGPRs across the wave: contact i's constants and impulses in lane i, island body k's
    // velocity in lane k.  The Gauss-Seidel order is unchanged (one contact after another): for
    // contact i every lane reads the two bodies' velocities with v_readlane and evaluates its own
    // contact's update from its own registers, lane i's result is kept (impulses by a lane select,
    // velocities by v_readlane + v_writelane into the body lanes), so the iters x nc contact
    // updates never wait on LDS.  Float operations and their order are those
    // of solver_velocity, so the result is bitwise identical.  Every thread of the wave calls it;
    // needs is.nc <= 64.
    __device__ __forceinline__ static float rdl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
    __device__ __forceinline__ static int rdli(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
    // lane l of `old` replaced by the wave-uniform x (v_writelane_b32)
    __device__ __forceinline__ static float wrl(float old, float x, int l) { return __int_as_float(mrp_writelane(__float_as_int(x), l, __float_as_int(old))); }
    // lane l's value of a per-lane condition, wave-uniform (ballot + bit test: no readlane)
    __device__ __forceinline__ static bool lane_bit(bool c, int l) { return (__builtin_amdgcn_ballot_w64(c) >> l) & 1ull; }
    // Early exit, exact: one sweep is a pure function of (body velocities, contact impulses), so
    // once the state after sweep k equals the state after sweep k-2 bit for bit the sequence has
    // period 1 or 2 from there on and the state after sweep `iters` is the state after sweep k
    // whenever k and iters have the same parity.  The state is compared at the k with
    // iters - k = 0 mod 4 against a snapshot taken two sweeps earlier (every fourth sweep rather
    // than every second: the comparison is off the sweeps' dependency chain but not free).
    // envs whose islands reach 5-8 contacts (several blocks, or 5 agents: Heavy-v0 +5.9 % in the driver
    // window, profiles/r3g_ab_envs_1_2_5.txt) get scheduled sweeps for those too
    static constexpr bool SCHED_WIDE = NB > 1 || NA >= 5;
    // islands of NC = 3 or 4 contacts (the slowest lanes' islands): the contacts' bodies and point
    // counts are read out of their lanes once, before the sweeps, into scalar registers, and the
    // contact loop is unrolled, so a contact update issues no readlane for its schedule and the body
    // readlanes take a lane select written long before (no wait states); same operations and order as
    // the generic loop below
    template <int NC>
    MRP_LANES_FN int lanes_sweeps(Isl& is, VC* vcs, int iters, bool early_exit) {
        const int me = tid < NC ? tid : 0;
        CC my = load_cc(vcs[me]);
        const int cia = vcs[me].iaI, cib = vcs[me].ibI;
        const int bk = tid < is.nb ? tid : 0;
        float bvx = is.vvx[bk], bvy = is.vvy[bk], bw = is.vw[bk];
        int ia[NC], ib[NC], pc[NC];
#pragma unroll
        for (int i = 0; i < NC; ++i) { ia[i] = rdli(cia, i); ib[i] = rdli(cib, i); pc[i] = rdli(my.pcount, i); }
        auto sweep = [&] {
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                P2 vA = p2(rdl(bvx, ia[i]), rdl(bvy, ia[i])); float wA = rdl(bw, ia[i]);
                P2 vB = p2(rdl(bvx, ib[i]), rdl(bvy, ib[i])); float wB = rdl(bw, ib[i]);
                P2 ni, ti;
                vel_update(my, pc[i], PickLane{i}, ni, ti, vA, wA, vB, wB);
                if (tid == i) { my.ni = ni; my.ti = ti; }
                bvx = wrl(bvx, rdl(vA.x, i), ia[i]); bvy = wrl(bvy, rdl(vA.y, i), ia[i]); bw = wrl(bw, rdl(wA, i), ia[i]);
                bvx = wrl(bvx, rdl(vB.x, i), ib[i]); bvy = wrl(bvy, rdl(vB.y, i), ib[i]); bw = wrl(bw, rdl(wB, i), ib[i]);
            }
        };
        // MRP_LANES_PAIRS: two sweeps per loop trip, as sweep_pairs (an odd count runs its first sweep
        // alone); the exit bookkeeping then runs once per pair
        constexpr int STEP = MRP_LANES_PAIRS ? 2 : 1;
        int sweeps = 0;
        if (STEP == 2 && (iters & 1)) { sweep(); sweeps = 1; }
        P2 sni = my.ni, sti = my.ti;
        float sbx = bvx, sby = bvy, sbw = bw;
        bool have = ((iters - sweeps) & 3) == 2;   // the start is a snapshot point
        while (sweeps < iters) {
            sweep();
            if (STEP == 2) sweep();
            sweeps += STEP;
            const int left = iters - sweeps, m = exit_mask(sweeps);
            if (early_exit && (left & m) == 0 && have) {
                const uint32_t d = (__float_as_uint(my.ni.x) ^ __float_as_uint(sni.x)) | (__float_as_uint(my.ni.y) ^ __float_as_uint(sni.y)) |
                                   (__float_as_uint(my.ti.x) ^ __float_as_uint(sti.x)) | (__float_as_uint(my.ti.y) ^ __float_as_uint(sti.y)) |
                                   (__float_as_uint(bvx) ^ __float_as_uint(sbx)) | (__float_as_uint(bvy) ^ __float_as_uint(sby)) |
                                   (__float_as_uint(bw) ^ __float_as_uint(sbw));
                if (__builtin_amdgcn_ballot_w64(d != 0u) == 0) break;
            }
            if (early_exit && (left & m) == 2) {
                sni = my.ni; sti = my.ti; sbx = bvx; sby = bvy; sbw = bw;
                have = true;
            }
        }
        if (tid < is.nb) { is.vvx[tid] = bvx; is.vvy[tid] = bvy; is.vw[tid] = bw; }
        if (tid < NC) store_cc(vcs[tid], my);
        return sweeps;
    }
    __device__ __forceinline__ int solver_velocity_lanes(Isl& is, VC* vcs, int iters, bool early_exit = true) {
        {
            const int n = __builtin_amdgcn_readfirstlane(is.nc);
            if (n == 3) return lanes_sweeps<3>(is, vcs, iters, early_exit);
            if (n == 4) return lanes_sweeps<4>(is, vcs, iters, early_exit);
            if constexpr (SCHED_WIDE) {   // islands of 5-8 contacts (the 3-block config: +4 %)
                if (n == 5) return lanes_sweeps<5>(is, vcs, iters, early_exit);
                if (n == 6) return lanes_sweeps<6>(is, vcs, iters, early_exit);
                if (n == 7) return lanes_sweeps<7>(is, vcs, iters, early_exit);
                if (n == 8) return lanes_sweeps<8>(is, vcs, iters, early_exit);
            }
        }
        const int nc = is.nc;
        CC my = load_cc(vcs[tid < nc ? tid : 0]);   // lanes >= nc evaluate a copy of contact 0 and are never kept
        const int cia = vcs[tid < nc ? tid : 0].iaI, cib = vcs[tid < nc ? tid : 0].ibI;
        const int bk = tid < is.nb ? tid : 0;
        float bvx = is.vvx[bk], bvy = is.vvy[bk], bw = is.vw[bk];
        // state snapshot for the period check (taken at sweeps k with k = iters mod 2)
        P2 sni = my.ni, sti = my.ti;
        float sbx = bvx, sby = bvy, sbw = bw;
        bool have = snap_initial(iters);   // sweep 0 is a snapshot point
        const int ncu = __builtin_amdgcn_readfirstlane(nc);
        int sweeps = 0;
        for (int it = 0; it < iters; ++it) {
            ++sweeps;
            for (int i = 0; i < ncu; ++i) {
                // every lane evaluates ITS contact's update from contact i's body velocities;
                // only lane i's result is kept (the Gauss-Seidel order is contact by contact)
                const int ia = rdli(cia, i), ib = rdli(cib, i), pcount = rdli(my.pcount, i);
                P2 vA = p2(rdl(bvx, ia), rdl(bvy, ia)); float wA = rdl(bw, ia);
                P2 vB = p2(rdl(bvx, ib), rdl(bvy, ib)); float wB = rdl(bw, ib);
                P2 ni, ti;
                // the block solver's case is decided by lane i's values (wave-uniform branches);
                // the other lanes follow lane i's case and are discarded
                vel_update(my, pcount, PickLane{i}, ni, ti, vA, wA, vB, wB);
                if (tid == i) { my.ni = ni; my.ti = ti; }
                // lane i's results go to the lanes of bodies A and B (A first, as the reference stores)
                bvx = wrl(bvx, rdl(vA.x, i), ia); bvy = wrl(bvy, rdl(vA.y, i), ia); bw = wrl(bw, rdl(wA, i), ia);
                bvx = wrl(bvx, rdl(vB.x, i), ib); bvy = wrl(bvy, rdl(vB.y, i), ib); bw = wrl(bw, rdl(wB, i), ib);
            }
            const int left = iters - (it + 1), m = exit_mask(it + 1);   // snapshot at left = 2, compare at left = 0 (mod m + 1; see exit_mask)
            if (early_exit && (left & m) == 0 && have) {
                const uint32_t d = (__float_as_uint(my.ni.x) ^ __float_as_uint(sni.x)) | (__float_as_uint(my.ni.y) ^ __float_as_uint(sni.y)) |
                                   (__float_as_uint(my.ti.x) ^ __float_as_uint(sti.x)) | (__float_as_uint(my.ti.y) ^ __float_as_uint(sti.y)) |
                                   (__float_as_uint(bvx) ^ __float_as_uint(sbx)) | (__float_as_uint(bvy) ^ __float_as_uint(sby)) |
                                   (__float_as_uint(bw) ^ __float_as_uint(sbw));
                if (__builtin_amdgcn_ballot_w64(d != 0u) == 0) break;
            }
            if (early_exit && (left & m) == 2) {
                sni = my.ni; sti = my.ti; sbx = bvx; sby = bvy; sbw = bw;
                have = true;
            }
        }
        if (tid < is.nb) { is.vvx[tid] = bvx; is.vvy[tid] = bvy; is.vw[tid] = bw; }
        if (tid < nc) store_cc(vcs[tid], my);
        return sweeps;
    }

    // Register-resident sweeps for islands of one or two contacts (nine in ten islands of a v0
    // rollout have one, most of the rest two): every lane runs the same contact updates on the
    // same values, so the bodies' velocities and the impulses stay in registers through all the
    // sweeps - no readlane / writelane traffic - and the block solver's case tests are
    // wave-uniform branches (ballot of identical lanes).  Same float operations in the same order
    // as solver_velocity, same exact early exit as solver_velocity_lanes.
    __device__ __forceinline__ static bool uni(bool c) { return __builtin_amdgcn_ballot_w64(c) != 0; }
    // The block solver's case tests `a && b` as the wave-uniform decision.  PickUni: identical lanes
    // (register paths); PickLane: lane i's values (lanes path).  `both` takes the two compares apart,
    // so each ballot is the v_cmp's own lane mask (no bool materialised in a VGPR and compared back)
    // and lane i's bit is one scalar bit test.
    struct PickUni {
        static constexpr bool LANES = false;
        __device__ __forceinline__ bool operator()(bool c) const { return uni(c); }
        __device__ __forceinline__ bool both(bool a, bool b) const {
#if MRP_VEL_PICK2
            return (__builtin_amdgcn_ballot_w64(a) & __builtin_amdgcn_ballot_w64(b)) != 0ull;
#else
            return uni(a && b);
#endif
        }
    };
    struct PickLane {
        static constexpr bool LANES = true;
        int i;
        __device__ __forceinline__ bool operator()(bool c) const { return lane_bit(c, i); }
        __device__ __forceinline__ bool both(bool a, bool b) const {
#if MRP_VEL_PICK2
            return ((__builtin_amdgcn_ballot_w64(a) & __builtin_amdgcn_ballot_w64(b)) >> i) & 1ull;
#else
            return lane_bit(a && b, i);
#endif
        }
    };
    // One contact's velocity-constraint constants (VC) in registers, as packed pairs (P2: one
    // v_pk_* instruction for both halves of a b2Vec2 operation) and the impulses (the state).
    struct CC {
        P2 rA0, rB0, rA1, rB1;   // arms of points 0 and 1, stored as pperp(r) = (-r.y, r.x) (see pcrossp)
        P2 normal, k01, k13, nm01, nm13;   // K = [k0 k1; k1 k3], K^-1 = [nm0 nm1; nm1 nm3]
        // no velocity bias: every fixture of these envs has restitution 0 (checked at mrp_create), so
        // SolveVelocityConstraints' velocityBias is -0 * vRel = +0 or the initial +0, and vn - (+0) == vn
        // bit for bit (-0 - +0 = -0): the subtraction is dropped, not approximated
        P2 mA, mB;   // (mA, mA), (mB, mB): broadcast once, not re-splatted (and hoisted into extra pairs) per use
        float nmass0, nmass1, tmass0, tmass1, iA, iB, friction;
        int pcount;
        P2 ni, ti;   // normal / tangent impulses of points 0 and 1
    };
    __device__ __forceinline__ static CC load_cc(const VC& c) {
        CC o;
        o.rA0 = p2(-c.rAy[0], c.rAx[0]); o.rB0 = p2(-c.rBy[0], c.rBx[0]);
        o.rA1 = p2(-c.rAy[1], c.rAx[1]); o.rB1 = p2(-c.rBy[1], c.rBx[1]);
        o.normal = p2(c.nx, c.ny);
        o.k01 = p2(c.k0, c.k1); o.k13 = p2(c.k1, c.k3);  o.nm01 = p2(c.nm0, c.nm1); o.nm13 = p2(c.nm1, c.nm3);
        o.nmass0 = c.nmass[0]; o.nmass1 = c.nmass[1]; o.tmass0 = c.tmass[0]; o.tmass1 = c.tmass[1];
        o.mA = pbc(c.mA); o.iA = c.iA; o.mB = pbc(c.mB); o.iB = c.iB; o.friction = c.friction;
        o.pcount = c.pointCount;
        o.ni = p2(c.ni[0], c.ni[1]); o.ti = p2(c.ti[0], c.ti[1]);
        return o;
    }
    __device__ __forceinline__ static void store_cc(VC& c, const CC& o) { c.ni[0] = o.ni.x; c.ni[1] = o.ni.y; c.ti[0] = o.ti.x; c.ti[1] = o.ti.y; }
    // b2ContactSolver::SolveVelocityConstraints for one contact, with the float operations and
    // order of solver_velocity (each packed half is the scalar expression, see P2 in mrp_math.h).
    // `pcount` is wave-uniform; `pick(c)` turns the block solver's per-lane case condition into the
    // wave-uniform decision (uni: identical lanes; lane_bit: lane i's).  Reads the impulses from
    // c.ni / c.ti and returns the new ones in ni / ti (the caller decides which lanes keep them).
    // runtime point count (the lanes path: contact i's count, wave-uniform): one branch to the
    // compile-time forms
    template <class Pick>
    __device__ __forceinline__ static void vel_update(const CC& c, int pcount, Pick pick, P2& ni, P2& ti,
                                                          P2& vA, float& wA, P2& vB, float& wB) {
        if (pcount == 2) vel_update_t<2>(c, pick, ni, ti, vA, wA, vB, wB);
        else vel_update_t<1>(c, pick, ni, ti, vA, wA, vB, wB);
    }
    // PCOUNT = the contact's manifold point count, a template parameter so every branch on it is
    // resolved at compile time (straight-line update, no phi copies between point-count paths)
    template <int PCOUNT, class Pick>
    __device__ __forceinline__ static void vel_update_t(const CC& c, Pick pick, P2& ni, P2& ti,
                                                            P2& vA, float& wA, P2& vB, float& wB) {
        vel_update_m<PCOUNT>(c, c.mA, c.iA, c.mB, c.iB, pick, ni, ti, vA, wA, vB, wB);
    }
    // the same with the two bodies' inverse masses / inertias passed in (equal to c.mA .. c.iB: the
    // solver copies them from the bodies), so a path that holds them per body need not per contact
    template <int PCOUNT, class Pick>
    __device__ __forceinline__ static void vel_update_m(const CC& c, const P2 mA, const float iA, const P2 mB, const float iB,
                                                            Pick pick, P2& ni, P2& ti, P2& vA, float& wA, P2& vB, float& wB) {
        constexpr int pcount = PCOUNT;
        // tangent = b2Cross(normal, 1.0f) = (1*n.y, -1*n.x) = (n.y, -n.x) exactly: a half swap and a
        // negation, which fold into the packed instructions' op_sel / neg modifiers
        const P2 normal = c.normal, tangent = p2(normal.y, -normal.x);
        ni = c.ni; ti = c.ti;
        {   // friction, point 0
            const P2 dv = ((vB + (pbc(wB) * c.rB0)) - vA) - (pbc(wA) * c.rA0);
            const float vt = MRP_VT(dv, normal, tangent);
            float lambda = c.tmass0 * (-vt);
            const float maxFriction = c.friction * ni.x;
            const float newImpulse = fclamp(ti.x + lambda, -maxFriction, maxFriction);
            lambda = newImpulse - ti.x;
            ti.x = newImpulse;
            const P2 P = MRP_PT(lambda, normal, tangent);
            vA = vA - mA * P;
            wA -= iA * pcrossp(c.rA0, P);
            vB = vB + mB * P;
            wB += iB * pcrossp(c.rB0, P);
        }
        if (pcount == 2) {   // friction, point 1
            const P2 dv = ((vB + (pbc(wB) * c.rB1)) - vA) - (pbc(wA) * c.rA1);
            const float vt = MRP_VT(dv, normal, tangent);
            float lambda = c.tmass1 * (-vt);
            const float maxFriction = c.friction * ni.y;
            const float newImpulse = fclamp(ti.y + lambda, -maxFriction, maxFriction);
            lambda = newImpulse - ti.y;
            ti.y = newImpulse;
            const P2 P = MRP_PT(lambda, normal, tangent);
            vA = vA - mA * P;
            wA -= iA * pcrossp(c.rA1, P);
            vB = vB + mB * P;
            wB += iB * pcrossp(c.rB1, P);
        }
        if (pcount == 1) {
            const P2 dv = ((vB + (pbc(wB) * c.rB0)) - vA) - (pbc(wA) * c.rA0);
            const float vn = pdot(dv, normal);
            float lambda = -c.nmass0 * vn;   // vn - velocityBias, velocityBias == +0 (see CC)
            const float newImpulse = fmax_(ni.x + lambda, 0.0f);
            lambda = newImpulse - ni.x;
            ni.x = newImpulse;
            const P2 P = pbc(lambda) * normal;
            vA = vA - mA * P;
            wA -= iA * pcrossp(c.rA0, P);
            vB = vB + mB * P;
            wB += iB * pcrossp(c.rB0, P);
        } else {
            const P2 a = ni;
            const P2 dv1 = ((vB + (pbc(wB) * c.rB0)) - vA) - (pbc(wA) * c.rA0);
            const P2 dv2 = ((vB + (pbc(wB) * c.rB1)) - vA) - (pbc(wA) * c.rA1);
            float vn1 = pdot(dv1, normal), vn2 = pdot(dv2, normal);
            // b = (vn1 - vbias0, vn2 - vbias1) - (k0*a.x + k2*a.y, k1*a.x + k3*a.y), k2 = k1, vbias == +0
            P2 b = p2(vn1, vn2);
            b = b - (c.k01 * pbc(a.x) + c.k13 * pbc(a.y));
            // x = -(nm0*b.x + nm2*b.y, nm1*b.x + nm3*b.y), nm2 = nm1
            // (not (-nm0)*b.x + (-nm1)*b.y: an exact cancellation gives +0 there where -(...) gives -0, and
            // the stored impulse would differ in its sign bit; measured, round 5)
            P2 x = -(c.nm01 * pbc(b.x) + c.nm13 * pbc(b.y));
            // Box2D's block solver applies the impulse of the first case that holds (both points
            // active, point 1 only, point 2 only, none), or none at all
            auto apply = [&](const P2 xs) {
                const P2 d = xs - a;
                const P2 P1 = pbc(d.x) * normal, P2v = pbc(d.y) * normal;
                const P2 S = P1 + P2v;
                vA = vA - mA * S;
                wA -= iA * (pcrossp(c.rA0, P1) + pcrossp(c.rA1, P2v));
                vB = vB + mB * S;
                wB += iB * (pcrossp(c.rB0, P1) + pcrossp(c.rB1, P2v));
                ni = xs;
            };
            if constexpr (MRP_VEL_BFREE && (!MRP_VEL_BFREE_LANES || Pick::LANES)) {
                // All four cases evaluated at once and the first that holds picked by selects, in Box2D's
                // order (both points active; point 1 only; point 2 only; none), so no case test waits on
                // the one before it.  The launches' slowest lanes mostly run the later cases (v0: 72 %
                // of their 2-point updates, v2: all; oracle b2o_lcp_cases on the captured lane-steps),
                // which the case-by-case branches reach only after one to three failed tests.
                const float x2 = -c.nmass0 * b.x, v2 = c.k01.y * x2 + b.y;   // case 2: x = (x2, 0), vn2 = k1 x2 + b.y
                const float x3 = -c.nmass1 * b.y, v3 = c.k01.y * x3 + b.x;   // case 3: x = (0, x3), vn1 = k1 x3 + b.x
                const bool c1 = x.x >= 0.0f && x.y >= 0.0f, c2 = x2 >= 0.0f && v2 >= 0.0f, c3 = x3 >= 0.0f && v3 >= 0.0f;
                P2 xs;
                xs.x = c1 ? x.x : (c2 ? x2 : 0.0f);
                xs.y = c1 ? x.y : (c2 ? 0.0f : (c3 ? x3 : 0.0f));
                // whether any case holds picked per lane as well: the impulse is applied unconditionally and
                // each output selected between the applied and the incoming value (the same bits either
                // way), so no ballot -> scalar -> branch sits on the chain.  Every lane decides from its
                // own values, which is the decision the kept lane needs (PickUni: identical lanes;
                // PickLane: lane i keeps contact i's own result)
                const bool any = c1 || c2 || c3 || (b.x >= 0.0f && b.y >= 0.0f);
                const P2 vA0 = vA, vB0 = vB, ni0 = ni;
                const float wA0 = wA, wB0 = wB;
                apply(xs);
                vA.x = any ? vA.x : vA0.x; vA.y = any ? vA.y : vA0.y; wA = any ? wA : wA0;
                vB.x = any ? vB.x : vB0.x; vB.y = any ? vB.y : vB0.y; wB = any ? wB : wB0;
                ni.x = any ? ni.x : ni0.x; ni.y = any ? ni.y : ni0.y;
                (void)pick;
            } else {
                bool ok = true;
                if (!pick.both(x.x >= 0.0f, x.y >= 0.0f)) {
                    x.x = -c.nmass0 * b.x; x.y = 0.0f;
                    vn2 = c.k01.y * x.x + b.y;
                    if (!pick.both(x.x >= 0.0f, vn2 >= 0.0f)) {
                        x.x = 0.0f; x.y = -c.nmass1 * b.y;
                        vn1 = c.k01.y * x.y + b.x;
                        if (!pick.both(x.y >= 0.0f, vn1 >= 0.0f)) {
                            x.x = 0.0f; x.y = 0.0f;
                            ok = pick.both(b.x >= 0.0f, b.y >= 0.0f);
                        }
                    }
                }
                if (ok) apply(x);
            }
        }
    }
    // the register-resident form: identical lanes, every lane keeps the result
    template <int PC>
    __device__ __forceinline__ static void cc_update(CC& c, P2& vA, float& wA, P2& vB, float& wB) {
        // opaque to the optimiser once per update, so values derived from the normal (the tangent,
        // its swapped / negated forms) are formed inside the instructions rather than hoisted out
        // of the sweep loop into registers of their own
        asm volatile("" : "+v"(c.normal));
        P2 ni, ti;
        vel_update_t<PC>(c, PickUni{}, ni, ti, vA, wA, vB, wB);
        c.ni = ni; c.ti = ti;
    }
    // exact early exit (see solver_velocity_lanes): the state after sweep k is compared with the
    // snapshot of sweep k-2 at every sweep k with iters - k = 0 mod 4, the snapshot is taken at
    // iters - k = 2 mod 4; true = the remaining sweeps are no-ops.  The comparison is one OR-tree
    // of XORs of the bit patterns (wave-uniform values: any lane decides).
    // The snapshot is held lane-distributed (value k in lane k of ONE register): the sweep state of
    // the register-resident paths is wave-uniform, so lane k can stand for all of value k, and the
    // snapshot costs one VGPR instead of NS (the sweeps' register peak sets k_step's spills).
    template <int NS> struct Snap {
        static_assert(NS <= 64, "one lane per snapshot value");
        float s;
        bool have;
        __device__ __forceinline__ static float gather(const float (&cur)[NS]) {
            float v = cur[0];
#pragma unroll
            for (int k = 1; k < NS; ++k) v = wrl(v, __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(cur[k]))), k);
            return v;
        }
        __device__ __forceinline__ Snap(const float (&cur)[NS], bool h) : s(gather(cur)), have(h) {}
        __device__ __forceinline__ void take(const float (&cur)[NS]) { s = gather(cur); have = true; }
        __device__ __forceinline__ bool same(const float (&cur)[NS]) const {
            const bool diff = (int)threadIdx.x < NS && __float_as_uint(gather(cur)) != __float_as_uint(s);
            return have && __builtin_amdgcn_ballot_w64(diff) == 0;
        }
        // one early-exit point after sweep `it + 1` of `iters`
        __device__ __forceinline__ bool step(int it, int iters, const float (&cur)[NS]) {
            const int left = iters - (it + 1), m = exit_mask(it + 1);
            if ((left & m) == 0) return same(cur);
            if ((left & m) == 2) take(cur);
            return false;
        }
    };
    // The early-exit schedule: after sweep k (left = iters - k) the state is compared with the
    // snapshot taken two sweeps earlier when left = 0 mod M, and a snapshot is taken when
    // left = 2 mod M, with M = 4 for the first EXIT_DENSE sweeps and M = EXIT_SPARSE after
    // (both powers of two, so a compare point of either phase has its snapshot exactly two sweeps
    // before it: left + 2 = 2 mod 4 and mod M).  Any such schedule exits exactly (the state then
    // has period 1 or 2 and iters - k is even); most islands that repeat do so within a few
    // sweeps, and the islands that never repeat (the launch's slowest lanes) pay the snapshot and
    // compare once per M sweeps instead of once per 4.
    static constexpr int EXIT_DENSE = 32, EXIT_SPARSE = 16;   // profiles/r4_ab_sparse_exit.txt
    static_assert(EXIT_SPARSE >= 4 && (EXIT_SPARSE & (EXIT_SPARSE - 1)) == 0, "a power of two >= 4");
    __device__ __forceinline__ static int exit_mask(int done) { return done > EXIT_DENSE ? EXIT_SPARSE - 1 : 3; }
    __device__ __forceinline__ static bool snap_initial(int iters) { return (iters & 3) == 2; }   // sweep 0 is a snapshot point
    // The sweep loop of the register paths: `sweep()` runs one Gauss-Seidel sweep, `state(v)` names
    // the NS values of the sweep state.  Every compare point has iters - k even, so the sweeps run in
    // pairs and the loop carries no per-sweep parity test or exit bookkeeping (an odd count runs its
    // first sweep alone); returns the sweeps run.
    template <int NS, class Sweep, class State>
    __device__ __forceinline__ static int sweep_pairs(int iters, bool early_exit, Sweep sweep, State state) {
        int it = 0;
        if (iters & 1) { sweep(); it += 1; }
        float cur[NS];
        state(cur);
        Snap<NS> snap(cur, ((iters - it) & 3) == 2);
        while (it < iters) {
            sweep();
            sweep();
            it += 2;
            if (early_exit) {
                state(cur);
                if (snap.step(it - 1, iters, cur)) break;
            }
        }
        return it;
    }
    // register paths: the contacts' point counts (wave-uniform, fixed for the whole solve) select a
    // compile-time instantiation of the sweep loop
    __device__ __forceinline__ int solver_velocity_one(Isl& is, VC* vcs, int iters, bool early_exit = true) {
        return __builtin_amdgcn_readfirstlane(vcs[0].pointCount) == 2 ? sweep_one<2>(is, vcs, iters, early_exit)
                                                                       : sweep_one<1>(is, vcs, iters, early_exit);
    }
    template <int P0>
    MRP_SOLVE_FN int sweep_one(Isl& is, VC* vcs, int iters, bool early_exit) {
        CC c = load_cc(vcs[0]);
        const int ia = vcs[0].iaI, ib = vcs[0].ibI;
        P2 vA = p2(is.vvx[ia], is.vvy[ia]); float wA = is.vw[ia];
        P2 vB = p2(is.vvx[ib], is.vvy[ib]); float wB = is.vw[ib];
        const int sweeps = sweep_pairs<10>(iters, early_exit, [&] { cc_update<P0>(c, vA, wA, vB, wB); }, [&](float (&v)[10]) {
            v[0] = vA.x; v[1] = vA.y; v[2] = wA; v[3] = vB.x; v[4] = vB.y; v[5] = wB; v[6] = c.ni.x; v[7] = c.ni.y; v[8] = c.ti.x; v[9] = c.ti.y;
        });
        if (tid == 0) {
            is.vvx[ia] = vA.x; is.vvy[ia] = vA.y; is.vw[ia] = wA;
            is.vvx[ib] = vB.x; is.vvy[ib] = vB.y; is.vw[ib] = wB;
            store_cc(vcs[0], c);
        }
        return sweeps;
    }
    // Two contacts: an island of two contacts has three bodies, X shared by both contacts, Y the
    // other body of contact 0 and Z that of contact 1; X's role (A or B) in each contact is a
    // template parameter, so every body access is a register.
    template <bool XA0, bool XA1, int P0, int P1>
    MRP_SOLVE_FN int sweep_two(Isl& is, VC* vcs, int iters, bool early_exit, int x, int y, int z) {
        CC c0 = load_cc(vcs[0]), c1 = load_cc(vcs[1]);
        P2 vX = p2(is.vvx[x], is.vvy[x]), vY = p2(is.vvx[y], is.vvy[y]), vZ = p2(is.vvx[z], is.vvy[z]);
        float wX = is.vw[x], wY = is.vw[y], wZ = is.vw[z];
        const int sweeps = sweep_pairs<17>(iters, early_exit, [&] {
            if (XA0) cc_update<P0>(c0, vX, wX, vY, wY); else cc_update<P0>(c0, vY, wY, vX, wX);
            if (XA1) cc_update<P1>(c1, vX, wX, vZ, wZ); else cc_update<P1>(c1, vZ, wZ, vX, wX);
        }, [&](float (&v)[17]) {
            v[0] = vX.x; v[1] = vX.y; v[2] = wX; v[3] = vY.x; v[4] = vY.y; v[5] = wY; v[6] = vZ.x; v[7] = vZ.y; v[8] = wZ;
            v[9] = c0.ni.x; v[10] = c0.ni.y; v[11] = c0.ti.x; v[12] = c0.ti.y; v[13] = c1.ni.x; v[14] = c1.ni.y; v[15] = c1.ti.x; v[16] = c1.ti.y;
        });
        if (tid == 0) {   // contact 1 stores last, as the reference's per-contact write-back order leaves it
            is.vvx[x] = vX.x; is.vvy[x] = vX.y; is.vw[x] = wX;
            is.vvx[y] = vY.x; is.vvy[y] = vY.y; is.vw[y] = wY;
            is.vvx[z] = vZ.x; is.vvy[z] = vZ.y; is.vw[z] = wZ;
            store_cc(vcs[0], c0); store_cc(vcs[1], c1);
        }
        return sweeps;
    }
    // Two contacts between the same two bodies (e.g. an agent against both boxes of the T block):
    // contact 1 is (P, Q) when SAME, else (Q, P).
    template <bool SAME, int P0, int P1>
    MRP_SOLVE_FN int sweep_same(Isl& is, VC* vcs, int iters, bool early_exit, int p, int q) {
        CC c0 = load_cc(vcs[0]), c1 = load_cc(vcs[1]);
        P2 vP = p2(is.vvx[p], is.vvy[p]), vQ = p2(is.vvx[q], is.vvy[q]);
        float wP = is.vw[p], wQ = is.vw[q];
        const int sweeps = sweep_pairs<14>(iters, early_exit, [&] {
            cc_update<P0>(c0, vP, wP, vQ, wQ);
            if (SAME) cc_update<P1>(c1, vP, wP, vQ, wQ); else cc_update<P1>(c1, vQ, wQ, vP, wP);
        }, [&](float (&v)[14]) {
            v[0] = vP.x; v[1] = vP.y; v[2] = wP; v[3] = vQ.x; v[4] = vQ.y; v[5] = wQ;
            v[6] = c0.ni.x; v[7] = c0.ni.y; v[8] = c0.ti.x; v[9] = c0.ti.y; v[10] = c1.ni.x; v[11] = c1.ni.y; v[12] = c1.ti.x; v[13] = c1.ti.y;
        });
        if (tid == 0) {
            is.vvx[p] = vP.x; is.vvy[p] = vP.y; is.vw[p] = wP;
            is.vvx[q] = vQ.x; is.vvy[q] = vQ.y; is.vw[q] = wQ;
            store_cc(vcs[0], c0); store_cc(vcs[1], c1);
        }
        return sweeps;
    }
    // returns -1 when the two contacts share no body (cannot happen inside one island; the caller
    // then uses solver_velocity_lanes)
    template <int P0, int P1>
    __device__ __forceinline__ int solver_velocity_two_p(Isl& is, VC* vcs, int iters, bool early_exit) {
        const int a0 = vcs[0].iaI, b0 = vcs[0].ibI, a1 = vcs[1].iaI, b1 = vcs[1].ibI;
        if (a0 == a1 && b0 == b1) return sweep_same<true, P0, P1>(is, vcs, iters, early_exit, a0, b0);
        if (a0 == b1 && b0 == a1) return sweep_same<false, P0, P1>(is, vcs, iters, early_exit, a0, b0);
        if (a0 == a1) return sweep_two<true, true, P0, P1>(is, vcs, iters, early_exit, a0, b0, b1);
        if (a0 == b1) return sweep_two<true, false, P0, P1>(is, vcs, iters, early_exit, a0, b0, a1);
        if (b0 == a1) return sweep_two<false, true, P0, P1>(is, vcs, iters, early_exit, b0, a0, b1);
        if (b0 == b1) return sweep_two<false, false, P0, P1>(is, vcs, iters, early_exit, b0, a0, a1);
        return -1;
    }
    __device__ __forceinline__ int solver_velocity_two(Isl& is, VC* vcs, int iters, bool early_exit = true) {
        const int p0 = __builtin_amdgcn_readfirstlane(vcs[0].pointCount), p1 = __builtin_amdgcn_readfirstlane(vcs[1].pointCount);
        if (p0 == 2) return p1 == 2 ? solver_velocity_two_p<2, 2>(is, vcs, iters, early_exit)
                                    : solver_velocity_two_p<2, 1>(is, vcs, iters, early_exit);
        return p1 == 2 ? solver_velocity_two_p<1, 2>(is, vcs, iters, early_exit)
                       : solver_velocity_two_p<1, 1>(is, vcs, iters, early_exit);
    }

    // ---------------------------------------------------------------- lane-distributed position iterations
    // b2ContactSolver::SolvePositionConstraints (toi = false) or SolveTOIPositionConstraints
    // (toi = true), repeated until the reference's exit test passes or `iters` passes have run,
    // with the island held in VGPRs across the wave as in solver_velocity_lanes: contact i's
    // constants in lane i, island body k's position (c, a) in lane k, contact by contact in
    // Gauss-Seidel order with lane i's result kept.  The rotations come from a two-entry memo
    // keyed by the angle's bit pattern (b2Rot::Set is a pure function of the angle, and a body
    // with invI = 0 - the v0 agents, the walls - keeps its angle through every pass).  Returns
    // the number of passes run (the reference's loop count).  Every thread calls it; nc <= 64.
    // Rotations as packed (c, s) pairs: pmul_rv(q, v) = q * v.x + pperp(q) * v.y (see P2).
    __device__ __forceinline__ static P2 rot_cs(float angle) { const Rot q = rot(angle); return p2(q.c, q.s); }
    __device__ __forceinline__ static P2 prot(P2 q, P2 v) { return q * pbc(v.x) + pperp(q) * pbc(v.y); }
    // Rotation memo of the position passes: an angle of +0 (a static body's island angle) is answered
    // directly, other angles from two entries keyed by the bit pattern, the least recently used one
    // replaced on a miss (an agent with invI = 0 keeps its entry while the block's angle changes at
    // every point: 3 b2Rot::Set per pass fewer than round-robin on a 3-contact agent-block-wall island)
    struct RotMemo {
        uint32_t k0 = 0u, k1 = 0u;
        P2 q0 = {1.0f, 0.0f}, q1 = {1.0f, 0.0f};
        bool next1 = false;
        __device__ __forceinline__ P2 get(float angle) {
            const uint32_t b = __float_as_uint(angle);
            if (b == 0u) return p2(1.0f, 0.0f);   // +0 (every static body's island angle): b2Rot::Set(+0) = {s +0, c 1}
            if (b == k0) { next1 = true; return q0; }   // least recently used entry is replaced
            if (b == k1) { next1 = false; return q1; }
            const P2 q = rot_cs(angle);
            if (next1) { k1 = b; q1 = q; } else { k0 = b; q0 = q; }
            next1 = !next1;
            return q;
        }
    };
    // Register-resident position passes for islands of one or two contacts (the topologies of
    // solver_velocity_one / _two): every lane runs the same point updates on the same values, so
    // the bodies' positions stay in registers, the rotation memo is wave-uniform and nothing goes
    // through readlane / writelane.  Same float operations in the same order as solver_position.
    struct UniMemo {   // RotMemo with wave-uniform (identical-lane) angles: scalar branches
        uint32_t k0 = 0u, k1 = 0u;
        P2 q0 = {1.0f, 0.0f}, q1 = {1.0f, 0.0f};
        bool next1 = false;
        __device__ __forceinline__ P2 get(float angle) {
            const uint32_t b = __float_as_uint(angle);
            if (uni(b == 0u)) return p2(1.0f, 0.0f);
            if (uni(b == k0)) { next1 = true; return q0; }
            if (uni(b == k1)) { next1 = false; return q1; }
            const P2 q = rot_cs(angle);
            if (next1) { k1 = b; q1 = q; } else { k0 = b; q0 = q; }
            next1 = !next1;
            return q;
        }
    };
    struct PCC {   // one contact's position-constraint constants (PC + masses), in registers, packed
        P2 lcA, lcB, ln, lp0, q0, q1;   // local centres, local normal, local plane point, local points 0 / 1
        P2 mA, mB;                      // (mA, mA), (mB, mB)
        float radA, radB, iA, iB;
        int pcount, type;
    };
    __device__ __forceinline__ static PCC load_pcc(const VC& vc, const PC& pc, bool toi, int toiA, int toiB) {
        PCC o;
        o.lcA = p2(pc.lcAx, pc.lcAy); o.lcB = p2(pc.lcBx, pc.lcBy);
        o.ln = p2(pc.lnx, pc.lny); o.lp0 = p2(pc.lpx0, pc.lpy0);
        o.q0 = p2(pc.lpx[0], pc.lpy[0]); o.q1 = p2(pc.lpx[1], pc.lpy[1]);
        o.radA = pc.rA; o.radB = pc.rB;
        float mA = vc.mA, iA = vc.iA, mB = vc.mB, iB = vc.iB;
        if (toi) {
            if (!(vc.iaI == toiA || vc.iaI == toiB)) { mA = 0.0f; iA = 0.0f; }
            if (!(vc.ibI == toiA || vc.ibI == toiB)) { mB = 0.0f; iB = 0.0f; }
        }
        o.mA = pbc(mA); o.iA = iA; o.mB = pbc(mB); o.iB = iB;
        o.pcount = pc.pointCount;
        o.type = pc.type;
        return o;
    }
    // b2ContactSolver::SolvePositionConstraints (SolveTOIPositionConstraints) for one contact, with
    // the float operations and order of solver_position (each packed half is the scalar
    // expression).  `rots(aA, aB, qA, qB)` gives the bodies' rotations, b2Rot::Set of their angles
    // (A then B per point, as the reference sets xfA.q then xfB.q); `onSep(sep)` sees each point's
    // separation.
    template <class Rots, class OnSep>
    __device__ __forceinline__ static void pos_update(const PCC& c, int pcount, int type, float baum, Rots&& rots,
                                                      OnSep onSep, P2& cA, float& aA, P2& cB, float& aB) {
        const P2 mA = c.mA, mB = c.mB;
        const float iA = c.iA, iB = c.iB;
        for (int j = 0; j < 2; ++j) {
            if (j == pcount) break;
            P2 qA, qB;
            rots(aA, aB, qA, qB);
            const P2 pA = cA - prot(qA, c.lcA), pB = cB - prot(qB, c.lcB);
            const P2 lp = j == 0 ? c.q0 : c.q1;
            P2 normal, point; float sep;
            if (type == MT_FACEA) {
                normal = prot(qA, c.ln);
                const P2 planePoint = prot(qA, c.lp0) + pA;
                const P2 clipPoint = prot(qB, lp) + pB;
                sep = pdot(clipPoint - planePoint, normal) - c.radA - c.radB;
                point = clipPoint;
            } else {
                normal = prot(qB, c.ln);
                const P2 planePoint = prot(qB, c.lp0) + pB;
                const P2 clipPoint = prot(qA, lp) + pA;
                sep = pdot(clipPoint - planePoint, normal) - c.radA - c.radB;
                point = clipPoint;
                normal = -normal;
            }
            const P2 rA = point - cA, rB = point - cB;
            onSep(sep);
            const float Cc = fclamp(baum * (sep + LINEAR_SLOP), -MAX_LINEAR_CORRECTION, 0.0f);
            const float rnA = pcross(rA, normal), rnB = pcross(rB, normal);
            const float K = mA.x + mB.x + iA * rnA * rnA + iB * rnB * rnB;
            const float impulse = K > 0.0f ? -Cc / K : 0.0f;
            const P2 Pv = pbc(impulse) * normal;
            cA = cA - mA * Pv;
            aA -= iA * pcross(rA, Pv);
            cB = cB + mB * Pv;
            aB += iB * pcross(rB, Pv);
        }
    }
    // the register-resident form: identical lanes, one wave-uniform rotation source
    template <class Rots>
    __device__ __forceinline__ static void pcc_update(const PCC& c, P2& cA, float& aA, P2& cB, float& aB, float& minSep,
                                                      float baum, Rots&& rots) {
        pos_update(c, c.pcount, c.type, baum, rots, [&minSep](float sep) { minSep = fmin_(minSep, sep); }, cA, aA, cB, aB);
    }
    // NC = 1: contact 0 on (P, Q).  NC = 2: SAMEB - both contacts on P, Q (contact 1 as (P, Q) if
    // XA1 else (Q, P)); otherwise X (= P) shared, Y (= Q) the other body of contact 0, Z of contact 1,
    // X's role in contact k given by XA0 / XA1.
    template <int NC, bool SAMEB, bool XA0, bool XA1>
    MRP_SOLVE_FN int pos_sweep(Isl& is, const VC* vcs, const PC* pcs, bool toi, int toiA, int toiB, int iters,
                                             int p, int q, int z) {
        PCC c0 = load_pcc(vcs[0], pcs[0], toi, toiA, toiB);
        PCC c1 = load_pcc(vcs[NC - 1], pcs[NC - 1], toi, toiA, toiB);
        // point counts and manifold types are wave-uniform: read into scalar registers once, not per pass
        c0.pcount = __builtin_amdgcn_readfirstlane(c0.pcount); c0.type = __builtin_amdgcn_readfirstlane(c0.type);
        c1.pcount = __builtin_amdgcn_readfirstlane(c1.pcount); c1.type = __builtin_amdgcn_readfirstlane(c1.type);
        P2 cP = p2(is.pcx[p], is.pcy[p]), cQ = p2(is.pcx[q], is.pcy[q]), cZ = p2(is.pcx[z], is.pcy[z]);
        float aP = is.pa[p], aQ = is.pa[q], aZ = is.pa[z];
        const float baum = toi ? TOI_BAUMGARTE : BAUMGARTE;
        const float exitSep = toi ? -1.5f * LINEAR_SLOP : -3.0f * LINEAR_SLOP;
        // one pass; `with(k, upd)` runs contact k's update `upd(rots)` with the rotations it chooses
        // (the choice is per contact, so each arm is straight-line code); returns the minimum separation
        auto pass = [&](auto&& with) {
            float minSep = 0.0f;
            if (NC == 1 || SAMEB) {
                if (XA0) with(0, [&](auto&& r) { pcc_update(c0, cP, aP, cQ, aQ, minSep, baum, r); });
                else with(0, [&](auto&& r) { pcc_update(c0, cQ, aQ, cP, aP, minSep, baum, r); });
                if (NC == 2) {
                    if (XA1) with(1, [&](auto&& r) { pcc_update(c1, cP, aP, cQ, aQ, minSep, baum, r); });
                    else with(1, [&](auto&& r) { pcc_update(c1, cQ, aQ, cP, aP, minSep, baum, r); });
                }
            } else {
                if (XA0) with(0, [&](auto&& r) { pcc_update(c0, cP, aP, cQ, aQ, minSep, baum, r); });
                else with(0, [&](auto&& r) { pcc_update(c0, cQ, aQ, cP, aP, minSep, baum, r); });
                if (XA1) with(1, [&](auto&& r) { pcc_update(c1, cP, aP, cZ, aZ, minSep, baum, r); });
                else with(1, [&](auto&& r) { pcc_update(c1, cZ, aZ, cP, aP, minSep, baum, r); });
            }
            return minSep;
        };
        int it = 0;
        UniMemo memo;
        while (it < iters) {
            ++it;
            const float minSep = pass([&memo](int, auto&& upd) {
                upd([&memo](float a, float b, P2& qa, P2& qb) { qa = memo.get(a); qb = memo.get(b); });
            });
            if (uni(minSep >= exitSep)) break;
        }
        if (tid == 0) {
            is.pcx[p] = cP.x; is.pcy[p] = cP.y; is.pa[p] = aP;
            is.pcx[q] = cQ.x; is.pcy[q] = cQ.y; is.pa[q] = aQ;
            if (NC == 2 && !SAMEB) { is.pcx[z] = cZ.x; is.pcy[z] = cZ.y; is.pa[z] = aZ; }
        }
        return it;
    }
    // position passes of a one- or two-contact island; -1 = other topology (use the lanes version)
    __device__ __forceinline__ int solver_position_small(Isl& is, const VC* vcs, const PC* pcs, bool toi, int toiA, int toiB,
                                                         int iters) {
        const int nc = __builtin_amdgcn_readfirstlane(is.nc);
        const int a0 = vcs[0].iaI, b0 = vcs[0].ibI;
        if (nc == 1) return pos_sweep<1, true, true, true>(is, vcs, pcs, toi, toiA, toiB, iters, a0, b0, b0);
        if (nc != 2) return -1;
        const int a1 = vcs[1].iaI, b1 = vcs[1].ibI;
        if (a0 == a1 && b0 == b1) return pos_sweep<2, true, true, true>(is, vcs, pcs, toi, toiA, toiB, iters, a0, b0, b0);
        if (a0 == b1 && b0 == a1) return pos_sweep<2, true, true, false>(is, vcs, pcs, toi, toiA, toiB, iters, a0, b0, b0);
        if (a0 == a1) return pos_sweep<2, false, true, true>(is, vcs, pcs, toi, toiA, toiB, iters, a0, b0, b1);
        if (a0 == b1) return pos_sweep<2, false, true, false>(is, vcs, pcs, toi, toiA, toiB, iters, a0, b0, a1);
        if (b0 == a1) return pos_sweep<2, false, false, true>(is, vcs, pcs, toi, toiA, toiB, iters, b0, a0, b1);
        if (b0 == b1) return pos_sweep<2, false, false, false>(is, vcs, pcs, toi, toiA, toiB, iters, b0, a0, a1);
        return -1;
    }

    // The lanes path's passes (solver_position_lanes, lanes_passes): `contact(with)` runs one pass, and
    // for contact i calls `with(i, upd)`, which runs the point updates `upd(rots)` with the rotations
    // of lane i's angles (wave-uniform) from the rotation memo; the island's positions live
    // lane-distributed in bx / by / ba.  Returns the passes run.
    template <class Contact>
    __device__ __forceinline__ int lanes_pass_loop(int iters, float exitSep, Contact&& contact) {
        int it = 0;
        RotMemo memo;
        while (it < iters) {
            ++it;
            // every lane evaluates ITS contact's point updates; the rotations are those of lane i's
            // angles (wave-uniform), and lane i's result is kept
            const float minSep = contact([&memo](int i, auto&& upd) {
                upd([&memo, i](float a, float b, P2& qa, P2& qb) { qa = memo.get(rdl(a, i)); qb = memo.get(rdl(b, i)); });
            });
            if (minSep >= exitSep) break;
        }
        return it;
    }
    // position passes of islands of NC = 3 or 4 contacts with the schedule (bodies, point counts,
    // manifold types) read out of the lanes once, before the passes (see lanes_sweeps)
    template <int NC>
    MRP_LANES_FN int lanes_passes(Isl& is, const VC* vcs, const PC* pcs, bool toi, int toiA, int toiB, int iters) {
        const int me = tid < NC ? tid : 0;
        const PCC my = load_pcc(vcs[me], pcs[me], toi, toiA, toiB);
        const int cia = vcs[me].iaI, cib = vcs[me].ibI;
        const int bk = tid < is.nb ? tid : 0;
        float bx = is.pcx[bk], by = is.pcy[bk], ba = is.pa[bk];
        const float baum = toi ? TOI_BAUMGARTE : BAUMGARTE;
        const float exitSep = toi ? -1.5f * LINEAR_SLOP : -3.0f * LINEAR_SLOP;
        int ia[NC], ib[NC], pc[NC], ty[NC];
#pragma unroll
        for (int i = 0; i < NC; ++i) { ia[i] = rdli(cia, i); ib[i] = rdli(cib, i); pc[i] = rdli(my.pcount, i); ty[i] = rdli(my.type, i); }
        const int it = lanes_pass_loop(iters, exitSep, [&](auto&& with) {
            float minSep = 0.0f;   // wave-uniform: lane i's separations in contact / point order
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                P2 cA = p2(rdl(bx, ia[i]), rdl(by, ia[i])); float aA = rdl(ba, ia[i]);
                P2 cB = p2(rdl(bx, ib[i]), rdl(by, ib[i])); float aB = rdl(ba, ib[i]);
                with(i, [&](auto&& rots) {
                    pos_update(my, pc[i], ty[i], baum, rots, [&minSep, i](float sep) { minSep = fmin_(minSep, rdl(sep, i)); },
                               cA, aA, cB, aB);
                });
                bx = wrl(bx, rdl(cA.x, i), ia[i]); by = wrl(by, rdl(cA.y, i), ia[i]); ba = wrl(ba, rdl(aA, i), ia[i]);
                bx = wrl(bx, rdl(cB.x, i), ib[i]); by = wrl(by, rdl(cB.y, i), ib[i]); ba = wrl(ba, rdl(aB, i), ib[i]);
            }
            return minSep;
        });
        if (tid < is.nb) { is.pcx[tid] = bx; is.pcy[tid] = by; is.pa[tid] = ba; }
        return it;
    }
    __device__ __forceinline__ int solver_position_lanes(Isl& is, const VC* vcs, const PC* pcs, bool toi, int toiA, int toiB, int iters) {
        // single-block envs only: in the 3-block config the scheduled passes measured slower (-2.7 %,
        // also with 5-8 contact islands scheduled; profiles/r3g_ab_env4_schedules.txt)
        if constexpr (NB == 1) {
            const int n = __builtin_amdgcn_readfirstlane(is.nc);
            if (n == 3) return lanes_passes<3>(is, vcs, pcs, toi, toiA, toiB, iters);
            if (n == 4) return lanes_passes<4>(is, vcs, pcs, toi, toiA, toiB, iters);
        }
        const int nc = is.nc;
        const int me = tid < nc ? tid : 0;   // lanes >= nc evaluate a copy of contact 0 and are never kept
        const PCC my = load_pcc(vcs[me], pcs[me], toi, toiA, toiB);
        const int cia = vcs[me].iaI, cib = vcs[me].ibI;
        const int bk = tid < is.nb ? tid : 0;
        float bx = is.pcx[bk], by = is.pcy[bk], ba = is.pa[bk];
        const float baum = toi ? TOI_BAUMGARTE : BAUMGARTE;
        const float exitSep = toi ? -1.5f * LINEAR_SLOP : -3.0f * LINEAR_SLOP;
        const int ncu = __builtin_amdgcn_readfirstlane(nc);
        const int it = lanes_pass_loop(iters, exitSep, [&](auto&& with) {
            float minSep = 0.0f;   // wave-uniform: lane i's separations in contact / point order
            for (int i = 0; i < ncu; ++i) {
                const int ia = rdli(cia, i), ib = rdli(cib, i), pcount = rdli(my.pcount, i), type = rdli(my.type, i);
                P2 cA = p2(rdl(bx, ia), rdl(by, ia)); float aA = rdl(ba, ia);
                P2 cB = p2(rdl(bx, ib), rdl(by, ib)); float aB = rdl(ba, ib);
                with(i, [&](auto&& rots) {
                    pos_update(my, pcount, type, baum, rots, [&minSep, i](float sep) { minSep = fmin_(minSep, rdl(sep, i)); },
                               cA, aA, cB, aB);
                });
                bx = wrl(bx, rdl(cA.x, i), ia); by = wrl(by, rdl(cA.y, i), ia); ba = wrl(ba, rdl(aA, i), ia);
                bx = wrl(bx, rdl(cB.x, i), ib); by = wrl(by, rdl(cB.y, i), ib); ba = wrl(ba, rdl(aB, i), ib);
            }
            return minSep;
        });
        if (tid < is.nb) { is.pcx[tid] = bx; is.pcy[tid] = by; is.pa[tid] = ba; }
        return it;
    }

    __device__ __forceinline__ void integrate_positions(Isl& is, float h) {
        for (int i = 0; i < is.nb; ++i) {
            V2 c = v2(is.pcx[i], is.pcy[i]); float a = is.pa[i];
            V2 v = v2(is.vvx[i], is.vvy[i]); float w = is.vw[i];
            V2 translation = vmul(h, v);
            if (vdot(translation, translation) > MAX_TRANSLATION_SQ) {
                float ratio = MAX_TRANSLATION / vlen(translation);
                v.x *= ratio; v.y *= ratio;
            }
            float rotation = h * w;
            if (rotation * rotation > MAX_ROTATION_SQ) {
                float ratio = MAX_ROTATION / fabsf(rotation);
                w *= ratio;
            }
            c = vadd(c, vmul(h, v));
            a += h * w;
            is.pcx[i] = c.x; is.pcy[i] = c.y; is.pa[i] = a;
            is.vvx[i] = v.x; is.vvy[i] = v.y; is.vw[i] = w;
        }
    }
    __device__ __forceinline__ void island_add_body(Isl& is, int b) { is.index[b] = is.nb; is.bodies[is.nb++] = b; }

    // b2Island::Solve (discrete step of one island), in three parts: island_pre and island_post
    // run on thread 0; the velocity iterations between them run on the whole wave
    // (solver_velocity_lanes), or on thread 0 over LDS when the island has more than 64 contacts.
    __device__ __forceinline__ void island_pre(Isl& is, float h, float dtRatio, VC* vcs, PC* pcs) {
        for (int i = 0; i < is.nb; ++i) {
            int b = is.bodies[i];
            if (is_dyn(b)) {
                V2 c = v2(S.cx[b], S.cy[b]); float a = S.a[b];
                V2 v = v2(S.vx[b], S.vy[b]); float w = S.w[b];
                S.c0x[b] = S.cx[b]; S.c0y[b] = S.cy[b]; S.a0[b] = S.a[b];
                V2 g = v2(1.0f * 0.0f, 1.0f * 0.0f);   // gravityScale * gravity (0,0)
                V2 acc = vadd(g, vmul(L.invMass[b], v2(S.fx[b], S.fy[b])));
                v = vadd(v, vmul(h, acc));
                w += h * L.invI[b] * S.tq[b];
                { float s = 1.0f / (1.0f + h * L.linDamp[b]); v.x *= s; v.y *= s; }
                w *= 1.0f / (1.0f + h * L.angDamp[b]);
                is.pcx[i] = c.x; is.pcy[i] = c.y; is.pa[i] = a; is.vvx[i] = v.x; is.vvy[i] = v.y; is.vw[i] = w;
            } else {
                V2 c = center(b);
                is.pcx[i] = c.x; is.pcy[i] = c.y; is.pa[i] = 0.0f; is.vvx[i] = 0.0f; is.vvy[i] = 0.0f; is.vw[i] = 0.0f;
            }
        }
        MRP_TRACE(12, is.nc);
        if (is.nc > 0) {
            solver_init(is, vcs, pcs, true, dtRatio);
            solver_init_velocity(is, vcs, pcs);
            solver_warm_start(is, vcs);
        }
    }
    // thread 0, after the velocity sweeps: store the impulses, integrate positions
    __device__ __forceinline__ void island_mid(Isl& is, float h, VC* vcs) {
        if (is.nc > 0) solver_store(is, vcs);
        integrate_positions(is, h);
    }
    // position iterations (whole wave; thread 0 over LDS past 64 contacts), posIters counted as
    // the reference's loop does
    __device__ __forceinline__ void island_position(Isl& is, VC* vcs, PC* pcs, int nc) {
        if (nc > 0 && nc <= 64) {
            int n = solver_position_small(is, vcs, pcs, false, -1, -1, 60);
            if (n < 0) n = solver_position_lanes(is, vcs, pcs, false, -1, -1, 60);
            if (tid == 0) S.posIters += n;
        } else if (tid == 0) {
            if (nc > 0) {
                for (int it = 0; it < 60; ++it) {
                    ++S.posIters;
                    if (solver_position(is, vcs, pcs, false, -1, -1)) break;
                }
            } else {
                ++S.posIters;   // an empty island's first position pass already reports solved
            }
        }
    }
    // thread 0: positions and velocities back to the bodies
    __device__ __forceinline__ void island_post(Isl& is) {
        for (int i = 0; i < is.nb; ++i) {
            int b = is.bodies[i];
            if (!is_dyn(b)) continue;   // static bodies are unchanged by construction (v = 0, invMass = 0)
            S.cx[b] = is.pcx[i]; S.cy[b] = is.pcy[i]; S.a[b] = is.pa[i];
            S.vx[b] = is.vvx[i]; S.vy[b] = is.vvy[i]; S.w[b] = is.vw[i];
            sync_transform(b);
        }
    }

    // b2World::Solve, cooperative (every thread of the wave calls it): thread 0 builds one island
    // at a time by DFS (body list = reverse creation order; contact edges in list order) and runs
    // its serial parts; the wave runs its velocity iterations.  Islands are solved in the
    // reference's order.  The trailing FindNewContacts is issued by world_step_coop.
    // b2World::Solve's island building, on the whole wave.  The contact list after collide_coop is its
    // snapshot (sh.clist, list order) less the contacts it destroyed (sh.cover = 0): no contact is
    // created or destroyed between the two.  Contact k of the list sits in lane k (and k + 64), with its
    // slot, its bodies and whether it may join an island (enabled and touching), so the reference's
    // walk of the whole list per popped body - a chain of dependent LDS loads on thread 0 - becomes one
    // ballot of the candidates, taken in list order (lowest lane first), which is the order the walk
    // meets them in.  The DFS stack is lane-distributed (entry j in lane j); the body flags, the stack
    // depth and the counts are wave-uniform.
    static constexpr int NLW = (C + 63) / 64;   // list words per lane
    __device__ __forceinline__ void solve_coop(float h, float dtRatio) {
        Isl& is = sh.isl;
        uint32_t bflag = 0;   // body island flags (bit per body), wave-uniform
        int seed = ND - 1;    // next DFS seed
        const int nl = sh.ccount;
        uint64_t joined[NLW];   // bit k: list contact k joined an island (CF_ISLAND), wave-uniform
#pragma unroll
        for (int w = 0; w < NLW; ++w) joined[w] = 0ull;
        for (int nisl = 0;; ++nisl) {
            MRP_PROG(0x3000u + nisl);
            refresh_tid();
            if (nisl > NBODY + 1) { if (tid == 0) S.fault = MRP_FAULT_ISLANDS; break; }
            while (seed >= 0 && (bflag & (1u << seed))) --seed;
            if (seed < 0) break;
            const unsigned long long td = MRP_NOW();
            int nb = 0, ncs = 0, sc = 0, stk = 0;
            uint32_t statics = 0u;
            stk = seed; sc = 1; bflag |= 1u << seed;
            // this lane's list contacts: slot, bodies, whether they may join an island (read per island,
            // so nothing of the list stays live in registers across the solver loops)
            int lslot[NLW], lA[NLW], lB[NLW];
            bool lok[NLW];
#pragma unroll
            for (int w = 0; w < NLW; ++w) {
                const int k = tid + 64 * w;
                const bool live = k < nl && sh.cover[k];
                const int c = live ? sh.clist[k] : 0;
                lslot[w] = c;
                lA[w] = live ? (int)L.fix_body[S.cfa[c]] : -1;
                lB[w] = live ? (int)L.fix_body[S.cfb[c]] : -1;
                const int f = live ? S.cflags[c] : 0;
                lok[w] = live && (f & CF_ENABLED) != 0 && (f & CF_TOUCHING) != 0;
            }
            for (int g = 0; sc > 0; ++g) {
                if (g > 2 * NBODY) { if (tid == 0) S.fault = MRP_FAULT_DFS; break; }
                const int b = __builtin_amdgcn_readlane(stk, sc - 1);
                --sc;
                if (tid == 0) { is.index[b] = nb; is.bodies[nb] = b; }   // island_add_body
                ++nb;
                if (!is_dyn(b)) { statics |= 1u << b; continue; }
#pragma unroll
                for (int w = 0; w < NLW; ++w) {
                    uint64_t m = __builtin_amdgcn_ballot_w64(lok[w] && (lA[w] == b || lB[w] == b)) & ~joined[w];
                    for (int q = 0; m != 0ull && q < 64; ++q) {
                        const int l = (int)__builtin_ctzll(m);
                        m &= m - 1ull;
                        if (ncs >= C || sc >= NBODY) { if (tid == 0) S.fault = MRP_FAULT_ISLAND_POOL; continue; }   // never in a valid world
                        const int c = __builtin_amdgcn_readlane(lslot[w], l);
                        const int other = __builtin_amdgcn_readlane(lA[w] == b ? lB[w] : lA[w], l);
                        if (tid == 0) is.contacts[ncs] = c;
                        ++ncs;
                        joined[w] |= 1ull << l;
                        if (bflag & (1u << other)) continue;
                        stk = mrp_writelane(other, sc, stk);
                        ++sc;
                        bflag |= 1u << other;
                    }
                }
            }
            if (tid == 0) {
                is.nb = nb; is.nc = ncs;
                MRP_SUB(32, td);
                const unsigned long long tp = MRP_NOW();
                island_pre(is, h, dtRatio, sh.u.sol.vcs, sh.u.sol.pcs);
                MRP_SUB(18, tp);
#ifdef MRP_STAMPS
                if ((uint32_t)is.nc > sh.trace[19]) sh.trace[19] = (uint32_t)is.nc;   // largest island's contacts
#endif
            }
            __syncthreads();
            const int nc = __builtin_amdgcn_readfirstlane(is.nc);
            const unsigned long long tv = MRP_NOW();
            // the lanes with the most contact updates set the kernel's duration: let their
            // sweeps win the SIMD's issue arbitration over co-resident waves
            const int lvl = nc >= 6 ? 3 : (nc >= 4 ? 2 : (nc >= 2 ? 1 : 0));
            if (nc > 0 && nc <= 64) {
                set_prio(lvl > step_prio ? lvl : step_prio);
                int sweeps = nc == 1 ? solver_velocity_one(is, sh.u.sol.vcs, 180) : (nc == 2 ? solver_velocity_two(is, sh.u.sol.vcs, 180) : -1);
                if (sweeps < 0) sweeps = solver_velocity_lanes(is, sh.u.sol.vcs, 180);
                MRP_TRACE(15, sweeps * nc);
                (void)sweeps;
            }
            else if (nc > 64 && tid == 0) for (int it = 0; it < 180; ++it) solver_velocity(is, sh.u.sol.vcs);
            MRP_SUB(16, tv);
            __syncthreads();
            MRP_PROG(0x3400u + nisl);
            if (tid == 0) { const unsigned long long tm = MRP_NOW(); island_mid(is, h, sh.u.sol.vcs); MRP_SUB(33, tm); }
            __syncthreads();
            MRP_PROG(0x3800u + nisl);
            const unsigned long long tq = MRP_NOW();
            island_position(is, sh.u.sol.vcs, sh.u.sol.pcs, nc);
            MRP_SUB(17, tq);
            if (nc > 0 && nc <= 64) set_prio(step_prio);
            __syncthreads();
            MRP_PROG(0x3c00u + nisl);
            if (tid == 0) {
                const unsigned long long tw = MRP_NOW();
                island_post(is);
                MRP_SUB(33, tw);
            }
            bflag &= ~statics;   // static bodies may join later islands
            --seed;
        }
        // the contacts that joined an island carry CF_ISLAND, as after the reference's walk (the flag is
        // cleared for every listed contact at the start of the solve and set on joining)
#pragma unroll
        for (int w = 0; w < NLW; ++w) {
            const int k = tid + 64 * w;
            if (k < nl && sh.cover[k]) {
                const int c = sh.clist[k];
                S.cflags[c] = ((joined[w] >> tid) & 1ull) ? (S.cflags[c] | CF_ISLAND) : (S.cflags[c] & ~CF_ISLAND);
            }
        }
        sync_fixtures_coop(bflag);
        __syncthreads();
    }

    // ---------------------------------------------------------------- TOI
    __device__ __forceinline__ SweepV sweep(int b, const float* salpha0) const {
        SweepV s;
        if (b < ND) { s.lcx = L.lcx[b]; s.lcy = L.lcy[b]; s.c0x = S.c0x[b]; s.c0y = S.c0y[b]; s.cx = S.cx[b]; s.cy = S.cy[b]; s.a0 = S.a0[b]; s.a = S.a[b]; s.alpha0 = S.alpha0[b]; }
        else { s.lcx = 0.0f; s.lcy = 0.0f; s.c0x = s.cx = L.wall_px[b - ND]; s.c0y = s.cy = L.wall_py[b - ND]; s.a0 = s.a = 0.0f; s.alpha0 = salpha0[b - ND]; }
        return s;
    }
    __device__ __forceinline__ static Xf sweep_xf(const SweepV& s, float beta) {
        Xf x;
        x.p = vadd(vmul(1.0f - beta, v2(s.c0x, s.c0y)), vmul(beta, v2(s.cx, s.cy)));
        float angle = (1.0f - beta) * s.a0 + beta * s.a;
        x.q = rot_z(angle);
        x.p = vsub(x.p, mul_rv(x.q, v2(s.lcx, s.lcy)));
        return x;
    }
    __device__ __forceinline__ static void sweep_advance(SweepV& s, float alpha) {
        float beta = (alpha - s.alpha0) / (1.0f - s.alpha0);
        V2 c0 = vadd(v2(s.c0x, s.c0y), vmul(beta, vsub(v2(s.cx, s.cy), v2(s.c0x, s.c0y))));
        s.c0x = c0.x; s.c0y = c0.y;
        s.a0 += beta * (s.a - s.a0);
        s.alpha0 = alpha;
    }
    __device__ __forceinline__ void sweep_store(int b, const SweepV& s, float* salpha0) {
        if (b < ND) { S.c0x[b] = s.c0x; S.c0y[b] = s.c0y; S.cx[b] = s.cx; S.cy[b] = s.cy; S.a0[b] = s.a0; S.a[b] = s.a; S.alpha0[b] = s.alpha0; }
        else salpha0[b - ND] = s.alpha0;
    }
    __device__ __forceinline__ void body_advance(int b, float alpha, float* salpha0) {   // b2Body::Advance
        SweepV s = sweep(b, salpha0);
        sweep_advance(s, alpha);
        s.cx = s.c0x; s.cy = s.c0y; s.a = s.a0;
        sweep_store(b, s, salpha0);
        if (b < ND) sync_transform(b);
    }

    __device__ __forceinline__ static int support(const DProxy& p, V2 d) {
        int best = 0; float bv = vdot(p.v[0], d);
        for (int i = 1; i < p.count; ++i) { float val = vdot(p.v[i], d); if (val > bv) { best = i; bv = val; } }
        return best;
    }
    // GJK simplex in named registers (an indexed array would live in scratch memory)
    __device__ __forceinline__ static SVert make_vert(const DProxy& pA, Xf xA, const DProxy& pB, Xf xB, int iA, int iB) {
        SVert v;
        v.iA = iA; v.iB = iB;
        v.wA = mul_xv(xA, pA.v[iA]); v.wB = mul_xv(xB, pB.v[iB]);
        v.w = vsub(v.wB, v.wA); v.a = 0.0f;
        return v;
    }
    __device__ __forceinline__ static float s_metric(const Simplex& s) {
        if (s.count == 2) return vlen(vsub(s.v0.w, s.v1.w));
        if (s.count == 3) return vcross(vsub(s.v1.w, s.v0.w), vsub(s.v2.w, s.v0.w));
        return 0.0f;
    }
    __device__ __forceinline__ static void s_solve2(Simplex& s) {
        V2 w1 = s.v0.w, w2 = s.v1.w, e12 = vsub(w2, w1);
        float d12_2 = -vdot(w1, e12);
        if (d12_2 <= 0.0f) { s.v0.a = 1.0f; s.count = 1; return; }
        float d12_1 = vdot(w2, e12);
        if (d12_1 <= 0.0f) { s.v1.a = 1.0f; s.count = 1; s.v0 = s.v1; return; }
        float inv = 1.0f / (d12_1 + d12_2);
        s.v0.a = d12_1 * inv; s.v1.a = d12_2 * inv; s.count = 2;
    }
    __device__ __forceinline__ static void s_solve3(Simplex& s) {
        V2 w1 = s.v0.w, w2 = s.v1.w, w3 = s.v2.w;
        V2 e12 = vsub(w2, w1);
        float d12_1 = vdot(w2, e12), d12_2 = -vdot(w1, e12);
        V2 e13 = vsub(w3, w1);
        float d13_1 = vdot(w3, e13), d13_2 = -vdot(w1, e13);
        V2 e23 = vsub(w3, w2);
        float d23_1 = vdot(w3, e23), d23_2 = -vdot(w2, e23);
        float n123 = vcross(e12, e13);
        float d123_1 = n123 * vcross(w2, w3), d123_2 = n123 * vcross(w3, w1), d123_3 = n123 * vcross(w1, w2);
        if (d12_2 <= 0.0f && d13_2 <= 0.0f) { s.v0.a = 1.0f; s.count = 1; return; }
        if (d12_1 > 0.0f && d12_2 > 0.0f && d123_3 <= 0.0f) { float inv = 1.0f / (d12_1 + d12_2); s.v0.a = d12_1 * inv; s.v1.a = d12_2 * inv; s.count = 2; return; }
        if (d13_1 > 0.0f && d13_2 > 0.0f && d123_2 <= 0.0f) { float inv = 1.0f / (d13_1 + d13_2); s.v0.a = d13_1 * inv; s.v2.a = d13_2 * inv; s.count = 2; s.v1 = s.v2; return; }
        if (d12_1 <= 0.0f && d23_2 <= 0.0f) { s.v1.a = 1.0f; s.count = 1; s.v0 = s.v1; return; }
        if (d13_1 <= 0.0f && d23_1 <= 0.0f) { s.v2.a = 1.0f; s.count = 1; s.v0 = s.v2; return; }
        if (d23_1 > 0.0f && d23_2 > 0.0f && d123_1 <= 0.0f) { float inv = 1.0f / (d23_1 + d23_2); s.v1.a = d23_1 * inv; s.v2.a = d23_2 * inv; s.count = 2; s.v0 = s.v2; return; }
        float inv = 1.0f / (d123_1 + d123_2 + d123_3);
        s.v0.a = d123_1 * inv; s.v1.a = d123_2 * inv; s.v2.a = d123_3 * inv; s.count = 3;
    }
    // b2Distance (GJK), returns distance between the (radius-free) cores
    __device__ __forceinline__ static float gjk(SCache& cache, const DProxy& pA, Xf xA, const DProxy& pB, Xf xB) {
        Simplex s;
        s.count = cache.count;
        s.v1.iA = s.v1.iB = s.v2.iA = s.v2.iB = -1;
        if (s.count > 0) s.v0 = make_vert(pA, xA, pB, xB, cache.iA0, cache.iB0);
        if (s.count > 1) s.v1 = make_vert(pA, xA, pB, xB, cache.iA1, cache.iB1);
        if (s.count > 2) s.v2 = make_vert(pA, xA, pB, xB, cache.iA2, cache.iB2);
        if (s.count > 1) {
            float m1 = cache.metric, m2 = s_metric(s);
            if (m2 < 0.5f * m1 || 2.0f * m1 < m2 || m2 < FLT_EPS) s.count = 0;
        }
        if (s.count == 0) {
            s.v0 = make_vert(pA, xA, pB, xB, 0, 0);
            s.v0.a = 1.0f; s.count = 1;
        }
        int iter = 0;
        while (iter < 20) {
            const int saveCount = s.count;
            const int sA0 = s.v0.iA, sB0 = s.v0.iB, sA1 = s.v1.iA, sB1 = s.v1.iB, sA2 = s.v2.iA, sB2 = s.v2.iB;
            if (s.count == 2) s_solve2(s); else if (s.count == 3) s_solve3(s);
            if (s.count == 3) break;
            V2 d;
            if (s.count == 1) d = vneg(s.v0.w);
            else {
                V2 e12 = vsub(s.v1.w, s.v0.w);
                float sgn = vcross(e12, vneg(s.v0.w));
                d = sgn > 0.0f ? vcross_sv(1.0f, e12) : vcross_vs(e12, 1.0f);
            }
            if (vlensq(d) < FLT_EPS * FLT_EPS) break;
            SVert vt;
            vt.iA = support(pA, mulT_rv(xA.q, vneg(d)));
            vt.wA = mul_xv(xA, pA.v[vt.iA]);
            vt.iB = support(pB, mulT_rv(xB.q, d));
            vt.wB = mul_xv(xB, pB.v[vt.iB]);
            vt.w = vsub(vt.wB, vt.wA);
            vt.a = 0.0f;
            ++iter;
            const bool dup = (vt.iA == sA0 && vt.iB == sB0) || (saveCount > 1 && vt.iA == sA1 && vt.iB == sB1) ||
                             (saveCount > 2 && vt.iA == sA2 && vt.iB == sB2);
            if (dup) break;
            if (s.count == 1) s.v1 = vt; else s.v2 = vt;
            ++s.count;
        }
        V2 pa = v2(0.0f, 0.0f), pb = v2(0.0f, 0.0f);
        if (s.count == 1) { pa = s.v0.wA; pb = s.v0.wB; }
        else if (s.count == 2) {
            pa = vadd(vmul(s.v0.a, s.v0.wA), vmul(s.v1.a, s.v1.wA));
            pb = vadd(vmul(s.v0.a, s.v0.wB), vmul(s.v1.a, s.v1.wB));
        } else if (s.count == 3) {
            pa = vadd(vadd(vmul(s.v0.a, s.v0.wA), vmul(s.v1.a, s.v1.wA)), vmul(s.v2.a, s.v2.wA));
            pb = pa;
        }
        float dist = vlen(vsub(pa, pb));
        cache.metric = s_metric(s); cache.count = s.count;
        cache.iA0 = s.v0.iA; cache.iB0 = s.v0.iB; cache.iA1 = s.v1.iA; cache.iB1 = s.v1.iB; cache.iA2 = s.v2.iA; cache.iB2 = s.v2.iB;
        return dist;
    }
    __device__ __forceinline__ static float sep_eval(const SepFn& f, const DProxy& pA, const DProxy& pB, const SweepV& sA, const SweepV& sB, int iA, int iB, float t) {
        Xf xA = sweep_xf(sA, t), xB = sweep_xf(sB, t);
        if (f.type == 0) return vdot(vsub(mul_xv(xB, pB.v[iB]), mul_xv(xA, pA.v[iA])), f.axis);
        if (f.type == 1) {
            V2 normal = mul_rv(xA.q, f.axis);
            V2 pointA = mul_xv(xA, f.lp);
            return vdot(vsub(mul_xv(xB, pB.v[iB]), pointA), normal);
        }
        V2 normal = mul_rv(xB.q, f.axis);
        V2 pointB = mul_xv(xB, f.lp);
        return vdot(vsub(mul_xv(xA, pA.v[iA]), pointB), normal);
    }
    __device__ __forceinline__ static float sep_min(const SepFn& f, const DProxy& pA, const DProxy& pB, const SweepV& sA, const SweepV& sB, int& iA, int& iB, float t) {
        Xf xA = sweep_xf(sA, t), xB = sweep_xf(sB, t);
        if (f.type == 0) {
            iA = support(pA, mulT_rv(xA.q, f.axis)); iB = support(pB, mulT_rv(xB.q, vneg(f.axis)));
            return vdot(vsub(mul_xv(xB, pB.v[iB]), mul_xv(xA, pA.v[iA])), f.axis);
        }
        if (f.type == 1) {
            V2 normal = mul_rv(xA.q, f.axis);
            V2 pointA = mul_xv(xA, f.lp);
            iA = -1; iB = support(pB, mulT_rv(xB.q, vneg(normal)));
            return vdot(vsub(mul_xv(xB, pB.v[iB]), pointA), normal);
        }
        V2 normal = mul_rv(xB.q, f.axis);
        V2 pointB = mul_xv(xB, f.lp);
        iB = -1; iA = support(pA, mulT_rv(xA.q, vneg(normal)));
        return vdot(vsub(mul_xv(xA, pA.v[iA]), pointB), normal);
    }
    // A box around one body's core over its sweep (beta in [0, 1]): every vertex sits at
    // p(beta) + R(angle(beta)) (v - lc), p linear between c0 and c.  A body whose angle is 0 at both ends
    // (static bodies, the v0 agents) has R = identity, so its vertex offsets bound it directly;
    // otherwise every vertex lies within max |v - lc| of p(beta).  Rounding moves the box by ulps.
    __device__ __forceinline__ static void sweep_box(const DProxy& p, const SweepV& s, V2& lo, V2& hi) {
        const float px0 = fmin_(s.c0x, s.cx), px1 = fmax_(s.c0x, s.cx), py0 = fmin_(s.c0y, s.cy), py1 = fmax_(s.c0y, s.cy);
        if (s.a0 == 0.0f && s.a == 0.0f) {
            float xlo = 3.0e38f, xhi = -3.0e38f, ylo = 3.0e38f, yhi = -3.0e38f;
            for (int k = 0; k < p.count; ++k) {
                const float rx = p.v[k].x - s.lcx, ry = p.v[k].y - s.lcy;
                xlo = fmin_(xlo, rx); xhi = fmax_(xhi, rx); ylo = fmin_(ylo, ry); yhi = fmax_(yhi, ry);
            }
            lo = v2(px0 + xlo, py0 + ylo); hi = v2(px1 + xhi, py1 + yhi);
        } else {
            float r2 = 0.0f;
            for (int k = 0; k < p.count; ++k) {
                const float rx = p.v[k].x - s.lcx, ry = p.v[k].y - s.lcy;
                r2 = fmax_(r2, rx * rx + ry * ry);
            }
            const float R = sqrtf(r2);
            lo = v2(px0 - R, py0 - R); hi = v2(px1 + R, py1 + R);
        }
    }
    // true when b2TimeOfImpact cannot report e_touching for this pair: it does so only at a time t1 whose
    // core distance (GJK's, >= the true distance up to rounding; or the separation function's, which at
    // t1 is at least GJK's distance) is within target + tolerance, and the sweep boxes are farther apart
    // than that plus a margin of 0.05 m (10 linear slops, far above any rounding of these coordinates).
    // NaN coordinates never skip.
    __device__ __forceinline__ static bool toi_far(const DProxy& pA, const SweepV& sA, const DProxy& pB, const SweepV& sB) {
        V2 aLo, aHi, bLo, bHi;
        sweep_box(pA, sA, aLo, aHi);
        sweep_box(pB, sB, bLo, bHi);
        const float gx = fmax_(fmax_(aLo.x - bHi.x, bLo.x - aHi.x), 0.0f);
        const float gy = fmax_(fmax_(aLo.y - bHi.y, bLo.y - aHi.y), 0.0f);
        const float target = fmax_(LINEAR_SLOP, pA.radius + pB.radius - 3.0f * LINEAR_SLOP);
        const float thr = target + 0.25f * LINEAR_SLOP + 0.05f;
        return gx * gx + gy * gy > thr * thr;
    }
    // b2TimeOfImpact; state 3 == e_touching
    __device__ __forceinline__ static TOIOut time_of_impact(const DProxy& pA, const DProxy& pB, SweepV sA, SweepV sB) {
        TOIOut out; out.state = 0; out.t = 1.0f;
        {   // b2Sweep::Normalize
            float twoPi = 2.0f * B2_PI;
            float d = twoPi * floorf(sA.a0 / twoPi); sA.a0 -= d; sA.a -= d;
            d = twoPi * floorf(sB.a0 / twoPi); sB.a0 -= d; sB.a -= d;
        }
        const float tMax = 1.0f;
        float totalRadius = pA.radius + pB.radius;
        float target = fmax_(LINEAR_SLOP, totalRadius - 3.0f * LINEAR_SLOP);
        float tolerance = 0.25f * LINEAR_SLOP;
        float t1 = 0.0f;
        int iter = 0;
        SCache cache; cache.count = 0; cache.metric = 0.0f;
        for (;;) {
            Xf xA = sweep_xf(sA, t1), xB = sweep_xf(sB, t1);
            float distance = gjk(cache, pA, xA, pB, xB);
            if (distance <= 0.0f) { out.state = 2; out.t = 0.0f; break; }
            if (distance < target + tolerance) { out.state = 3; out.t = t1; break; }
            SepFn f;
            if (cache.count == 1) {
                f.type = 0;
                f.axis = vsub(mul_xv(xB, pB.v[cache.iB0]), mul_xv(xA, pA.v[cache.iA0]));
                vnormalize(f.axis);
                f.lp = v2(0.0f, 0.0f);
            } else if (cache.iA0 == cache.iA1) {
                f.type = 2;
                V2 b1 = pB.v[cache.iB0], b2 = pB.v[cache.iB1];
                f.axis = vcross_vs(vsub(b2, b1), 1.0f);
                vnormalize(f.axis);
                V2 normal = mul_rv(xB.q, f.axis);
                f.lp = vmul(0.5f, vadd(b1, b2));
                V2 pointB = mul_xv(xB, f.lp);
                V2 pointA = mul_xv(xA, pA.v[cache.iA0]);
                float s = vdot(vsub(pointA, pointB), normal);
                if (s < 0.0f) f.axis = vneg(f.axis);
            } else {
                f.type = 1;
                V2 a1 = pA.v[cache.iA0], a2 = pA.v[cache.iA1];
                f.axis = vcross_vs(vsub(a2, a1), 1.0f);
                vnormalize(f.axis);
                V2 normal = mul_rv(xA.q, f.axis);
                f.lp = vmul(0.5f, vadd(a1, a2));
                V2 pointA = mul_xv(xA, f.lp);
                V2 pointB = mul_xv(xB, pB.v[cache.iB0]);
                float s = vdot(vsub(pointB, pointA), normal);
                if (s < 0.0f) f.axis = vneg(f.axis);
            }
            bool done = false;
            float t2 = tMax;
            int pushBackIter = 0;
            for (;;) {
                int iA, iB;
                float s2 = sep_min(f, pA, pB, sA, sB, iA, iB, t2);
                if (s2 > target + tolerance) { out.state = 4; out.t = tMax; done = true; break; }
                if (s2 > target - tolerance) { t1 = t2; break; }
                float s1 = sep_eval(f, pA, pB, sA, sB, iA, iB, t1);
                if (s1 < target - tolerance) { out.state = 1; out.t = t1; done = true; break; }
                if (s1 <= target + tolerance) { out.state = 3; out.t = t1; done = true; break; }
                int rootIter = 0;
                float a1 = t1, a2 = t2;
                for (;;) {
                    float t;
                    if (rootIter & 1) t = a1 + (target - s1) * (a2 - a1) / (s2 - s1);
                    else t = 0.5f * (a1 + a2);
                    ++rootIter;
                    float s = sep_eval(f, pA, pB, sA, sB, iA, iB, t);
                    if (fabsf(s - target) < tolerance) { t2 = t; break; }
                    if (s > target) { a1 = t; s1 = s; } else { a2 = t; s2 = s; }
                    if (rootIter == 50) break;
                }
                ++pushBackIter;
                if (pushBackIter == MAX_POLY) break;
            }
            ++iter;
            if (done) break;
            if (iter == 20) { out.state = 1; out.t = t1; break; }
        }
        return out;
    }

    // b2Island::SolveTOI
    // b2Island::SolveTOI, first part (thread 0): position pre-solve and velocity constraints
    __device__ __forceinline__ void island_toi_pre(Isl& is, int toiA, int toiB, VC* vcs, PC* pcs) {
        for (int i = 0; i < is.nb; ++i) {
            int b = is.bodies[i];
            if (is_dyn(b)) { is.pcx[i] = S.cx[b]; is.pcy[i] = S.cy[b]; is.pa[i] = S.a[b]; is.vvx[i] = S.vx[b]; is.vvy[i] = S.vy[b]; is.vw[i] = S.w[b]; }
            else { V2 c = center(b); is.pcx[i] = c.x; is.pcy[i] = c.y; is.pa[i] = 0.0f; is.vvx[i] = 0.0f; is.vvy[i] = 0.0f; is.vw[i] = 0.0f; }
        }
        solver_init(is, vcs, pcs, false, 1.0f);
        sh.toiIA = toiA; sh.toiIB = toiB;
        // the TOI position iterations run on the whole wave next (solve_toi_coop), then island_toi_mid
    }
    // thread 0, after the TOI position iterations: the pair's sweep start, velocity constraints
    __device__ __forceinline__ void island_toi_mid(Isl& is, VC* vcs, PC* pcs) {
        const int toiA = sh.toiIA, toiB = sh.toiIB;
        {
            int ba = is.bodies[toiA], bb = is.bodies[toiB];
            if (is_dyn(ba)) { S.c0x[ba] = is.pcx[toiA]; S.c0y[ba] = is.pcy[toiA]; S.a0[ba] = is.pa[toiA]; }
            if (is_dyn(bb)) { S.c0x[bb] = is.pcx[toiB]; S.c0y[bb] = is.pcy[toiB]; S.a0[bb] = is.pa[toiB]; }
        }
        solver_init_velocity(is, vcs, pcs);
        // the 180 velocity sweeps run on the whole wave next (solve_toi_coop), then island_toi_post
    }
    __device__ __forceinline__ void island_toi_post(Isl& is, float dt) {
        integrate_positions(is, dt);
        for (int i = 0; i < is.nb; ++i) {
            int b = is.bodies[i];
            if (!is_dyn(b)) continue;
            S.cx[b] = is.pcx[i]; S.cy[b] = is.pcy[i]; S.a[b] = is.pa[i];
            S.vx[b] = is.vvx[i]; S.vy[b] = is.vvy[i]; S.w[b] = is.vw[i];
            sync_transform(b);
        }
    }

    // b2World::SolveTOI, cooperative.  Each pass of the event loop: thread 0 walks the contact
    // list in order, applying the alpha0 synchronisation (which mutates sweeps exactly as the
    // reference's scan does) and snapshotting the sweeps of every contact whose TOI must be
    // computed; all threads then run b2TimeOfImpact on one candidate each; thread 0 takes the
    // minimum in list order and processes the event serially.
    __device__ __forceinline__ void toi_scan() {
        float* salpha0 = sh.salpha0;
        int tn = 0, np = 0;
        for (int c = S.cHead, g_ = 0; c != NULLN && list_ok(g_); c = S.cnext[c]) {
            if ((S.cflags[c] & CF_ENABLED) == 0) continue;
            if (S.ctoiCount[c] > MAX_SUBSTEPS) continue;
            if (S.cflags[c] & CF_TOI) { sh.plan[np] = -2; sh.pslot[np++] = c; continue; }
            int fa = S.cfa[c], fb = S.cfb[c];
            int bA = L.fix_body[fa], bB = L.fix_body[fb];
            bool collideA = !is_dyn(bA), collideB = !is_dyn(bB);   // no bullets in these envs
            if (!collideA && !collideB) continue;
            SweepV sA = sweep(bA, salpha0), sB = sweep(bB, salpha0);
            if (sA.alpha0 < sB.alpha0) { sweep_advance(sA, sB.alpha0); sweep_store(bA, sA, salpha0); }
            else if (sB.alpha0 < sA.alpha0) { sweep_advance(sB, sA.alpha0); sweep_store(bB, sB, salpha0); }
            sh.tcand[tn] = c; sh.u.toi.tsA[tn] = sA; sh.u.toi.tsB[tn] = sB;
            sh.plan[np] = tn; sh.pslot[np++] = c;
            ++tn;
        }
        sh.tn = tn; sh.np = np;
    }
    // The first pass's candidate scan on the whole wave.  At the start of b2World::SolveTOI every sweep's
    // alpha0 is 0 (solve_toi_coop sets them) and no listed contact carries CF_TOI, so toi_scan's sweep
    // synchronisation (sweep_advance when the two alpha0 differ) never fires and its per-contact work is
    // independent: lane k takes list contact k, and only the candidate numbering needs the list order
    // (a prefix count of the candidates' ballot).  Same candidates, same order, same sweeps as toi_scan.
    __device__ __forceinline__ void toi_scan_first() {
        if (tid == 0) {   // the list in order (FindNewContacts has put the new contacts at its head)
            int n = 0;
            for (int c = S.cHead, g_ = 0; c != NULLN && list_ok(g_); c = S.cnext[c]) sh.clist[n++] = c;
            sh.ccount = n;
        }
        __syncthreads();
        const int n = sh.ccount;
        int tn = 0;
        for (int k0 = 0; k0 < n; k0 += 64) {
            const int k = k0 + tid;
            bool cand = false;
            int c = 0, bA = 0, bB = 0;
            if (k < n) {
                c = sh.clist[k];
                if ((S.cflags[c] & CF_ENABLED) != 0 && S.ctoiCount[c] <= MAX_SUBSTEPS) {
                    bA = L.fix_body[S.cfa[c]]; bB = L.fix_body[S.cfb[c]];
                    cand = !is_dyn(bA) || !is_dyn(bB);   // no bullets in these envs
                }
            }
            const uint64_t m = __builtin_amdgcn_ballot_w64(cand);
            if (cand) {
                const int idx = tn + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                sh.tcand[idx] = c; sh.u.toi.tsA[idx] = sweep(bA, sh.salpha0); sh.u.toi.tsB[idx] = sweep(bB, sh.salpha0);
                sh.plan[idx] = idx; sh.pslot[idx] = c;
            }
            tn += (int)__popcll(m);
        }
        if (tid == 0) { sh.tn = tn; sh.np = tn; }
    }
    // returns true when an event was processed that needs FindNewContacts
    __device__ __forceinline__ void toi_event(float dt) {
        float* salpha0 = sh.salpha0;
        int minC = NULLN; float minAlpha = 1.0f;
        for (int k = 0; k < sh.np; ++k) {
            int c = sh.pslot[k];
            float alpha;
            if (sh.plan[k] == -2) alpha = S.ctoi[c];
            else {
                int i = sh.plan[k];
                float alpha0 = sh.u.toi.tsA[i].alpha0;   // both sweeps share alpha0 after the sync
                TOIOut o = sh.u.toi.tout[i];
                if (o.state == 3) alpha = fmin_(alpha0 + (1.0f - alpha0) * o.t, 1.0f);
                else alpha = 1.0f;
                S.ctoi[c] = alpha;
                S.cflags[c] |= CF_TOI;
            }
            if (alpha < minAlpha) { minC = c; minAlpha = alpha; }
        }
        sh.toi_fnc = 0;
        if (minC == NULLN || 1.0f - 10.0f * FLT_EPS < minAlpha) { sh.toi_done = 1; return; }
        ++S.toiEvents;
        int fa = S.cfa[minC], fb = S.cfb[minC];
        int bA = L.fix_body[fa], bB = L.fix_body[fb];
        SweepV back1 = sweep(bA, salpha0), back2 = sweep(bB, salpha0);
        body_advance(bA, minAlpha, salpha0);
        body_advance(bB, minAlpha, salpha0);
        contact_update(minC);
        S.cflags[minC] &= ~CF_TOI;
        ++S.ctoiCount[minC];
        if ((S.cflags[minC] & CF_ENABLED) == 0 || (S.cflags[minC] & CF_TOUCHING) == 0) {
            S.cflags[minC] &= ~CF_ENABLED;
            sweep_store(bA, back1, salpha0); sweep_store(bB, back2, salpha0);
            if (bA < ND) sync_transform(bA);
            if (bB < ND) sync_transform(bB);
            return;   // no FindNewContacts on this path (reference `continue`)
        }
        Isl& is = sh.isl;
        uint32_t bflag = 0;
        is.nb = 0; is.nc = 0;
        island_add_body(is, bA); island_add_body(is, bB);
        is.contacts[is.nc++] = minC;
        bflag |= (1u << bA) | (1u << bB);
        S.cflags[minC] |= CF_ISLAND;
        const int pair[2] = {bA, bB};
        for (int k = 0; k < 2; ++k) {
            int body = pair[k];
            if (!is_dyn(body)) continue;
            for (int c = S.cHead, g_ = 0; c != NULLN && list_ok(g_); c = S.cnext[c]) {
                int cA = L.fix_body[S.cfa[c]], cB = L.fix_body[S.cfb[c]];
                if (cA != body && cB != body) continue;
                if (is.nb == 2 * MAX_TOI_CONTACTS) break;
                if (is.nc == MAX_TOI_CONTACTS) break;
                if (is.nc >= C || is.nb >= NBODY) { S.fault = MRP_FAULT_ISLAND_POOL; break; }   // never in a valid world
                if (S.cflags[c] & CF_ISLAND) continue;
                int other = cA == body ? cB : cA;
                if (is_dyn(other)) continue;   // only static bodies join a TOI island here
                SweepV backup = sweep(other, salpha0);
                if (!(bflag & (1u << other))) body_advance(other, minAlpha, salpha0);
                contact_update(c);
                if ((S.cflags[c] & CF_ENABLED) == 0 || (S.cflags[c] & CF_TOUCHING) == 0) {
                    sweep_store(other, backup, salpha0);
                    if (other < ND) sync_transform(other);
                    continue;
                }
                S.cflags[c] |= CF_ISLAND;
                is.contacts[is.nc++] = c;
                if (bflag & (1u << other)) continue;
                bflag |= 1u << other;
                island_add_body(is, other);
            }
        }
        island_toi_pre(is, is.index[bA], is.index[bB], sh.u.sol.vcs, sh.u.sol.pcs);
        sh.toi_dt = (1.0f - minAlpha) * dt;
        sh.toi_solve = 1;   // velocity sweeps next (whole wave), then toi_event_post
    }
    // the rest of one TOI event after the island's velocity sweeps (thread 0)
    __device__ __forceinline__ void toi_event_post() {
        Isl& is = sh.isl;
        island_toi_post(is, sh.toi_dt);
        for (int i = 0; i < is.nb; ++i) {
            int body = is.bodies[i];
            if (!is_dyn(body)) continue;
            sync_fixtures(body);
            for (int c = S.cHead, g_ = 0; c != NULLN && list_ok(g_); c = S.cnext[c]) {
                int cA = L.fix_body[S.cfa[c]], cB = L.fix_body[S.cfb[c]];
                if (cA == body || cB == body) S.cflags[c] &= ~(CF_TOI | CF_ISLAND);
            }
        }
        sh.toi_fnc = 1;
    }
    __device__ __forceinline__ void solve_toi_coop(float dt) {
        if (tid == 0) {
#if MRP_FRESH_REGS
            // the zero made here (v_mov), not a copy of one made at k_step's entry: under v0's
            // iterative-ilp schedule those copies lived across the step in scratch
            float zero;
            asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
#else
            const float zero = 0.0f;
#endif
            for (int i = 0; i < 4; ++i) sh.salpha0[i] = zero;
            for (int b = 0; b < ND; ++b) S.alpha0[b] = zero;
            for (int c = S.cHead, g_ = 0; c != NULLN && list_ok(g_); c = S.cnext[c]) { S.cflags[c] &= ~(CF_TOI | CF_ISLAND); S.ctoiCount[c] = 0; S.ctoi[c] = 1.0f; }
            sh.toi_done = 0;
        }
        for (int pass = 0;; ++pass) {
            MRP_PROG(0x2000u + pass);
            refresh_tid();
            if (pass > (MAX_SUBSTEPS + 1) * C + 2) { if (tid == 0) S.fault = MRP_FAULT_TOI_PASSES; break; }
            const unsigned long long ts = MRP_NOW();
            const unsigned long long tsc = MRP_NOW();
            if (pass == 0) toi_scan_first();
            else if (tid == 0) toi_scan();
            MRP_SUB(35, tsc);
            __syncthreads();
            const int tn = sh.tn;
            for (int i = tid; i < tn; i += 64) {
                int c = sh.tcand[i];
                int fa = S.cfa[c], fb = S.cfb[c];
                DProxy pA = {L.shape[fa].v, L.shape[fa].count, L.shape[fa].radius};
                DProxy pB = {L.shape[fb].v, L.shape[fb].count, L.shape[fb].radius};
                const SweepV sA = sh.u.toi.tsA[i], sB = sh.u.toi.tsB[i];
                TOIOut o;
                o.state = 4; o.t = 1.0f;   // e_separated: what b2TimeOfImpact returns for such a pair
                if (!toi_far(pA, sA, pB, sB)) o = time_of_impact(pA, pB, sA, sB);
                sh.u.toi.tout[i] = o;
            }
            __syncthreads();
            MRP_SUB(20, ts);   // candidate scan + b2TimeOfImpact of every candidate (the slowest thread's)
            const unsigned long long te = MRP_NOW();
            MRP_PROG(0x2800u + pass);
            if (tid == 0) { sh.toi_solve = 0; toi_event(dt); }
            __syncthreads();
#ifdef MRP_STAMPS_TOI   // words 22 / 23: the event's thread-0 set-up, its sub-step solve (-DMRP_STAMPS -DMRP_STAMPS_TOI)
            MRP_SUB(22, te);
            const unsigned long long tsv = MRP_NOW();
#endif
            if (sh.toi_solve) {
                const int nc = __builtin_amdgcn_readfirstlane(sh.isl.nc);
                if (nc <= 64) {
                    set_prio(2 > step_prio ? 2 : step_prio);   // a TOI event is on this lane's critical path
                    if (solver_position_small(sh.isl, sh.u.sol.vcs, sh.u.sol.pcs, true, sh.toiIA, sh.toiIB, 20) < 0)
                        solver_position_lanes(sh.isl, sh.u.sol.vcs, sh.u.sol.pcs, true, sh.toiIA, sh.toiIB, 20);
                } else if (tid == 0) {
                    for (int i = 0; i < 20; ++i) if (solver_position(sh.isl, sh.u.sol.vcs, sh.u.sol.pcs, true, sh.toiIA, sh.toiIB)) break;
                }
                __syncthreads();
                if (tid == 0) island_toi_mid(sh.isl, sh.u.sol.vcs, sh.u.sol.pcs);
                __syncthreads();
                if (nc <= 64) {
                    int sweeps = nc == 1 ? solver_velocity_one(sh.isl, sh.u.sol.vcs, 180)
                                         : (nc == 2 ? solver_velocity_two(sh.isl, sh.u.sol.vcs, 180) : -1);
                    if (sweeps < 0) solver_velocity_lanes(sh.isl, sh.u.sol.vcs, 180);
                    set_prio(step_prio);
                }
                else if (tid == 0) for (int i = 0; i < 180; ++i) solver_velocity(sh.isl, sh.u.sol.vcs);
                __syncthreads();
#ifdef MRP_STAMPS_TOI
                MRP_SUB(23, tsv);
#endif
                if (tid == 0) toi_event_post();
                __syncthreads();
            }
            MRP_PROG(0x2c00u + pass);
            if (sh.toi_done) { MRP_SUB(21, te); break; }
            if (sh.toi_fnc) find_new_contacts_coop();
            MRP_SUB(21, te);   // the event: island, sub-step solve, FindNewContacts
        }
    }

    // b2World::Step(1/50, 180, 60), cooperative (every thread of the wave calls it)
    __device__ __forceinline__ void world_step_coop() {
        const float dt = 1.0f / 50;
        if (S.newFixture) {
            __syncthreads();
            if (tid == 0) S.newFixture = 0;
            find_new_contacts_coop();   // begins with a barrier-separated read of moveBuf
        }
        MRP_STAMP(2);
        float inv_dt = 1.0f / dt;
        float dtRatio = S.inv_dt0 * dt;
        collide_coop();
        MRP_STAMP(3);
        solve_coop(dt, dtRatio);
        MRP_STAMP(4);
        find_new_contacts_coop();
        MRP_STAMP(5);
        solve_toi_coop(dt);
        MRP_STAMP(6);
        if (tid == 0) {
            S.inv_dt0 = inv_dt;
            for (int b = 0; b < ND; ++b) { S.fx[b] = 0.0f; S.fy[b] = 0.0f; S.tq[b] = 0.0f; }
        }
        __syncthreads();
    }
};

}  // namespace mrp
