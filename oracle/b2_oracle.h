/*
 * b2_oracle.h -- TEST INFRASTRUCTURE ONLY (parity oracle; never linked into the product).
 *
 * Plain-C CPU restatement of the subset of Box2D v2.3.x (the engine vendored in the
 * third-party `box2d-py` wheel that gym_puzzles calls through pybox2d) that the
 * MultiRobotPuzzle step path exercises.  The engine source is NOT present in
 * /root/reference; this file restates the published v2.3.1
 * algorithms (pointer-linked lists, dynamic AABB tree, b2CollidePolygons, sequential
 * impulse contact solver with the 2-point block solver, island DFS, TOI via GJK +
 * conservative advancement) with the same float32 operation order, so that it can
 * serve as the CPU oracle the HIP kernels are checked against bit for bit.
 *
 * Parity with pybox2d itself is UNPINNED: no fixture in the reference pins a step
 * result and box2d-py cannot be imported here.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 */
#ifndef MRP_B2_ORACLE_H
#define MRP_B2_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y; } V2;
typedef struct { float s, c; } Rot;
typedef struct { V2 p; Rot q; } Xf;
typedef struct { V2 localCenter, c0, c; float a0, a, alpha0; } Sweep;
typedef struct { V2 lo, hi; } AABB;

#define B2_MAX_POLY 8
typedef struct { int count; V2 v[B2_MAX_POLY]; V2 n[B2_MAX_POLY]; V2 centroid; float radius; } Poly;

struct Body; struct Contact; struct World;

typedef struct Fixture {
    struct Fixture* next;
    struct Body* body;
    Poly shape;
    float density, friction, restitution;
    int proxyId;
    AABB aabb;          /* b2FixtureProxy::aabb */
    int tag;            /* env-level fixture index */
} Fixture;

typedef struct ContactEdge {
    struct Body* other;
    struct Contact* contact;
    struct ContactEdge* prev;
    struct ContactEdge* next;
} ContactEdge;

enum { BT_STATIC = 0, BT_KINEMATIC = 1, BT_DYNAMIC = 2 };
enum { BF_ISLAND = 1, BF_AWAKE = 2, BF_AUTOSLEEP = 4, BF_BULLET = 8, BF_FIXEDROT = 16, BF_ACTIVE = 32, BF_TOI = 64 };

typedef struct Body {
    int type, flags, islandIndex;
    Xf xf;
    Sweep sweep;
    V2 v; float w;
    V2 force; float torque;
    struct World* world;
    struct Body* prev; struct Body* next;
    Fixture* fixtureList; int fixtureCount;
    ContactEdge* contactList;
    float mass, invMass, I, invI;
    float linearDamping, angularDamping, gravityScale;
    int tag;            /* env-level body index */
} Body;

typedef struct { V2 localPoint; float normalImpulse, tangentImpulse; uint32_t id; } MPoint;
enum { MT_CIRCLES = 0, MT_FACEA = 1, MT_FACEB = 2 };
typedef struct { MPoint points[2]; V2 localNormal, localPoint; int type, pointCount; } Manifold;

enum { CF_ISLAND = 1, CF_TOUCHING = 2, CF_ENABLED = 4, CF_FILTER = 8, CF_BULLETHIT = 16, CF_TOI = 32 };
typedef struct Contact {
    int flags;
    struct Contact* prev; struct Contact* next;
    ContactEdge nodeA, nodeB;
    Fixture* fA; Fixture* fB;
    Manifold manifold;
    int toiCount; float toi;
    float friction, restitution, tangentSpeed;
} Contact;

typedef struct {
    AABB aabb; void* userData; int parent; /* == next in free list */
    int child1, child2, height;
} TreeNode;
typedef struct { int root; TreeNode* nodes; int nodeCount, nodeCapacity, freeList, insertionCount; int maxId; } Tree;
typedef struct { int a, b; } Pair;
typedef struct {
    Tree tree; int proxyCount;
    int* moveBuf; int moveCap, moveCount, maxMove;
    Pair* pairBuf; int pairCap, pairCount;
    int queryProxyId;
} BroadPhase;

typedef void (*ContactCb)(void* ctx, Contact* c);
typedef struct {
    BroadPhase bp;
    Contact* contactList; int contactCount, maxContacts;
    long satCalls;      /* work model: b2CollidePolygons calls (contact updates) */
    ContactCb begin, end; void* listenerCtx;   /* NULL begin/end == no listener */
} ContactManager;

/* Work model (test infrastructure, tools/chain_model.py): the serial solver work one lane's
 * step carries as the device runs it -- velocity sweeps counted with the device's exact early exit
 * (mrp_world.h solver_velocity_*: state after sweep k equals the state after k-2) -- and the same
 * work grouped into dependency levels (consecutive Gauss-Seidel contacts whose dynamic bodies are
 * disjoint commute bit-exactly).  Counts accumulate from world creation. */
typedef struct {
    long islands;                        /* discrete islands with >= 1 contact */
    long vel_sweeps;                     /* velocity sweeps run */
    long vel_upd1, vel_upd2;             /* contact updates run, 1- / 2-point */
    long vel_levels;                     /* sweeps run x dependency levels of the island */
    long pos_passes, pos_points;         /* position passes, point updates */
    long pos_level_points;               /* passes x sum over levels of the level's largest point count */
    long toi_vel_upd, toi_vel_levels;    /* the same for TOI islands */
    long toi_pos_points, toi_pos_level_points;
    long sat_calls, toi_calls;           /* narrow-phase polygon pairs, b2TimeOfImpact calls */
    long vel_pipe;                       /* critical path of the velocity sweeps (discrete + TOI islands) unrolled
                                          * over all sweeps run: contacts of sweep k+1 may start once the
                                          * contacts they share dynamic bodies with have finished */
    long pos_pipe;                       /* the same for the position passes, weighted by point count */
    long isl_units;                      /* discrete islands' velocity updates + position points */
    long isl_concurrent_save;            /* per step: those units minus the largest island's (what solving a
                                          * step's independent islands concurrently would take off the chain) */
    long vel_1wave, vel_2wave;           /* b2o_model_2wave (off: 0): modelled cycles of the discrete islands'
                                          * velocity sweeps on one wave, and split over two waves of one
                                          * workgroup (best contact partition, LDS handoffs priced) */
} OrWork;

enum { WF_NEWFIXTURE = 1, WF_LOCKED = 2, WF_CLEARFORCES = 4 };
typedef struct World {
    Body* bodyList; int bodyCount;
    ContactManager cm;
    float inv_dt0;
    int flags;
    int stepComplete;
    V2 gravity;
    /* diagnostics */
    long toiEvents, posIters, velIters;
    long touching;      /* touching contacts after each Step's Collide, summed (the device's counter) */
    /* capacity high-water marks (test infrastructure: the device keeps fixed per-lane pools,
     * tests/test_oracle.py checks these stay inside them) */
    int maxIslandBodies, maxIslandContacts, maxToiIslandBodies, maxToiIslandContacts;
    OrWork work;
    long stepIslSum, stepIslMax;         /* work model: this step's island units, sum and max */
} World;

typedef struct { int type; V2 position; float angle; float linearDamping, angularDamping; int tag; } BodyDef;
typedef struct { const Poly* shape; float density, friction, restitution; int tag; } FixtureDef;

/* shapes (b2PolygonShape) */
void b2o_poly_set(Poly* p, const V2* verts, int count);
void b2o_poly_box(Poly* p, float hx, float hy);
void b2o_poly_box_oriented(Poly* p, float hx, float hy, V2 center, float angle);
void b2o_poly_mass(const Poly* p, float density, float* mass, V2* center, float* I);

/* world */
World* b2o_world_create(void);
void b2o_world_destroy(World* w);
Body* b2o_create_body(World* w, const BodyDef* def);
Fixture* b2o_create_fixture(Body* b, const FixtureDef* def);
void b2o_destroy_body(World* w, Body* b);
void b2o_step(World* w, float dt, int velIters, int posIters);
void b2o_set_listener(World* w, ContactCb begin, ContactCb end, void* ctx);

/* diagnostic: period histogram of the islands whose velocity sweeps never reach period 1 or 2
 * (see b2_oracle.c); on >= 0 resets and sets the switch, out300 (may be NULL) receives it */
void b2o_period_diag(int on, long* out300);
/* diagnostic: the work model counts velocity sweeps as if periods up to p were detected (0 = the device) */
void b2o_model_period(int p);
/* diagnostic: price the velocity sweeps on one wave and split over two (OrWork vel_1wave /
 * vel_2wave); cost[(p - 1) * 8 + n - 1] = cycles of one p-point contact update on a wave holding n
 * contacts (n > 8 priced as 8), x = cycles of one cross-wave handoff, b = cycles of the two waves'
 * joint early-exit compare; cost NULL switches the model off */
void b2o_model_2wave(const double* cost16, double x, double b);
/* diagnostic: with factor > 0, vel_2wave prices the paired one-wave path instead (slots of one or two
 * same-point-count updates, b2o_dual_schedule, each priced as one update x factor); 0 switches it off */
void b2o_model_dual(double factor, int window);
/* the paired path's slot schedule of D sweeps of an nc-contact island (see b2_oracle.c) */
int b2o_dual_schedule(int nc, const int* ia, const int* ib, const int* dyn, const int* pcount, int D, int window,
                      unsigned char* out, int cap);
/* diagnostic: topology histogram of 3- and 4-contact islands (see b2_oracle.c) */
void b2o_topo_diag(int on, long* sig64, long* w64);

/* body API used by the env layer (pybox2d semantics) */
void b2o_set_linear_velocity(Body* b, V2 v);
void b2o_set_angular_velocity(Body* b, float w);
void b2o_apply_force(Body* b, V2 f, V2 point);
void b2o_apply_linear_impulse(Body* b, V2 j, V2 point);
void b2o_apply_angular_impulse(Body* b, float j);
void b2o_apply_torque(Body* b, float t);
V2 b2o_world_point(const Body* b, V2 local);
V2 b2o_world_vector(const Body* b, V2 local);
float b2o_inertia(const Body* b);

#ifdef __cplusplus
}
#endif
#endif
