/*
 * b2_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the Box2D v2.3.1 subset
 * used by gym_puzzles (see b2_oracle.h for scope and the "parity unpinned" caveat).
 *
 * Structure deliberately mirrors upstream Box2D (pointer-linked body/fixture/contact
 * lists, a dynamic AABB tree with a LIFO free list, a move buffer + sorted pair buffer)
 * so that contact ordering -- which decides Gauss-Seidel order and fixture A/B roles --
 * is reproduced the way pybox2d's engine produces it.  The HIP kernels in
 * gym_puzzles_amd/csrc are an independent, array-based restatement; agreement between
 * the two is what the parity tests check.
 *
 * Reference call sites this serves: world.Step(1/50, 180, 60) at
 * gym_puzzles/envs/multi_robot_puzzle_00.py:428 and multi_robot_puzzle_02.py:478;
 * body/fixture creation at multi_robot_puzzle_00.py:268,313-351,368 and
 * multi_robot_puzzle_02.py:322-341,363-389,402.
 *
 * Compile with -O2 -ffp-contract=off -fno-fast-math (IEEE float32, no FMA contraction),
 * matching how the box2d-py wheel's C++ is built for baseline x86-64.
 */
#include "b2_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- settings [B2 b2Settings.h] */
#define LINEAR_SLOP 0.005f
#define POLY_RADIUS (2.0f * LINEAR_SLOP)
#define AABB_EXT 0.1f
#define AABB_MUL 2.0f
#define MAX_TRANSLATION 2.0f
#define MAX_TRANSLATION_SQ (MAX_TRANSLATION * MAX_TRANSLATION)
#define B2_PI 3.14159265359f
#define MAX_ROTATION (0.5f * B2_PI)
#define MAX_ROTATION_SQ (MAX_ROTATION * MAX_ROTATION)
#define BAUMGARTE 0.2f
#define TOI_BAUMGARTE 0.75f
#define VELOCITY_THRESHOLD 1.0f
#define MAX_LINEAR_CORRECTION 0.2f
#define MAX_SUBSTEPS 8
#define MAX_TOI_CONTACTS 32
#define NULLN (-1)

/* ---------------------------------------------------------------- math [B2 b2Math.h] */
static inline V2 v2(float x, float y) { V2 r; r.x = x; r.y = y; return r; }
static inline V2 vadd(V2 a, V2 b) { return v2(a.x + b.x, a.y + b.y); }
static inline V2 vsub(V2 a, V2 b) { return v2(a.x - b.x, a.y - b.y); }
static inline V2 vmul(float s, V2 a) { return v2(s * a.x, s * a.y); }
static inline V2 vneg(V2 a) { return v2(-a.x, -a.y); }
static inline float vdot(V2 a, V2 b) { return a.x * b.x + a.y * b.y; }
static inline float vcross(V2 a, V2 b) { return a.x * b.y - a.y * b.x; }
static inline V2 vcross_vs(V2 a, float s) { return v2(s * a.y, -s * a.x); }
static inline V2 vcross_sv(float s, V2 a) { return v2(-s * a.y, s * a.x); }
static inline float vlen(V2 a) { return sqrtf(a.x * a.x + a.y * a.y); }
static inline float vlensq(V2 a) { return a.x * a.x + a.y * a.y; }
static inline float vnormalize(V2* a) {
    float length = sqrtf(a->x * a->x + a->y * a->y);
    if (length < FLT_EPSILON) return 0.0f;
    float inv = 1.0f / length;
    a->x *= inv; a->y *= inv;
    return length;
}
static inline float fmin_(float a, float b) { return a < b ? a : b; }
static inline float fmax_(float a, float b) { return a > b ? a : b; }
static inline float fclamp(float a, float lo, float hi) { return fmax_(lo, fmin_(a, hi)); }
static inline V2 vmin(V2 a, V2 b) { return v2(fmin_(a.x, b.x), fmin_(a.y, b.y)); }
static inline V2 vmax(V2 a, V2 b) { return v2(fmax_(a.x, b.x), fmax_(a.y, b.y)); }
static inline Rot rot(float angle) { Rot q; q.s = sinf(angle); q.c = cosf(angle); return q; }
static inline V2 mul_rv(Rot q, V2 v) { return v2(q.c * v.x - q.s * v.y, q.s * v.x + q.c * v.y); }
static inline V2 mulT_rv(Rot q, V2 v) { return v2(q.c * v.x + q.s * v.y, -q.s * v.x + q.c * v.y); }
static inline V2 mul_xv(Xf T, V2 v) {
    float x = (T.q.c * v.x - T.q.s * v.y) + T.p.x;
    float y = (T.q.s * v.x + T.q.c * v.y) + T.p.y;
    return v2(x, y);
}
static inline V2 mulT_xv(Xf T, V2 v) {
    float px = v.x - T.p.x, py = v.y - T.p.y;
    return v2(T.q.c * px + T.q.s * py, -T.q.s * px + T.q.c * py);
}
static inline Rot mulT_rr(Rot q, Rot r) { Rot o; o.s = q.c * r.s - q.s * r.c; o.c = q.c * r.c + q.s * r.s; return o; }
static inline Xf mulT_xx(Xf A, Xf B) { Xf C; C.q = mulT_rr(A.q, B.q); C.p = mulT_rv(A.q, vsub(B.p, A.p)); return C; }

static inline void sweep_get_transform(const Sweep* s, Xf* xf, float beta) {
    xf->p = vadd(vmul(1.0f - beta, s->c0), vmul(beta, s->c));
    float angle = (1.0f - beta) * s->a0 + beta * s->a;
    xf->q = rot(angle);
    xf->p = vsub(xf->p, mul_rv(xf->q, s->localCenter));
}
static inline void sweep_advance(Sweep* s, float alpha) {
    float beta = (alpha - s->alpha0) / (1.0f - s->alpha0);
    s->c0 = vadd(s->c0, vmul(beta, vsub(s->c, s->c0)));
    s->a0 += beta * (s->a - s->a0);
    s->alpha0 = alpha;
}
static inline void sweep_normalize(Sweep* s) {
    float twoPi = 2.0f * B2_PI;
    float d = twoPi * floorf(s->a0 / twoPi);
    s->a0 -= d; s->a -= d;
}

static inline AABB aabb_combine(AABB a, AABB b) { AABB r; r.lo = vmin(a.lo, b.lo); r.hi = vmax(a.hi, b.hi); return r; }
static inline float aabb_perimeter(AABB a) { float wx = a.hi.x - a.lo.x; float wy = a.hi.y - a.lo.y; return 2.0f * (wx + wy); }
static inline int aabb_contains(AABB a, AABB b) {
    int r = 1;
    r = r && a.lo.x <= b.lo.x; r = r && a.lo.y <= b.lo.y;
    r = r && b.hi.x <= a.hi.x; r = r && b.hi.y <= a.hi.y;
    return r;
}
static inline int aabb_overlap(AABB a, AABB b) {
    V2 d1 = vsub(b.lo, a.hi), d2 = vsub(a.lo, b.hi);
    if (d1.x > 0.0f || d1.y > 0.0f) return 0;
    if (d2.x > 0.0f || d2.y > 0.0f) return 0;
    return 1;
}

/* ---------------------------------------------------------------- polygon shape [B2 b2PolygonShape.cpp] */
static V2 compute_centroid(const V2* vs, int count) {
    V2 c = v2(0.0f, 0.0f);
    float area = 0.0f;
    V2 pRef = v2(0.0f, 0.0f);
    const float inv3 = 1.0f / 3.0f;
    for (int i = 0; i < count; ++i) {
        V2 p1 = pRef, p2 = vs[i], p3 = i + 1 < count ? vs[i + 1] : vs[0];
        V2 e1 = vsub(p2, p1), e2 = vsub(p3, p1);
        float D = vcross(e1, e2);
        float triangleArea = 0.5f * D;
        area += triangleArea;
        c = vadd(c, vmul(triangleArea * inv3, vadd(vadd(p1, p2), p3)));
    }
    float s = 1.0f / area;
    c.x *= s; c.y *= s;
    return c;
}

void b2o_poly_box(Poly* p, float hx, float hy) {
    p->count = 4;
    p->v[0] = v2(-hx, -hy); p->v[1] = v2(hx, -hy); p->v[2] = v2(hx, hy); p->v[3] = v2(-hx, hy);
    p->n[0] = v2(0.0f, -1.0f); p->n[1] = v2(1.0f, 0.0f); p->n[2] = v2(0.0f, 1.0f); p->n[3] = v2(-1.0f, 0.0f);
    p->centroid = v2(0.0f, 0.0f);
    p->radius = POLY_RADIUS;
}

void b2o_poly_box_oriented(Poly* p, float hx, float hy, V2 center, float angle) {
    b2o_poly_box(p, hx, hy);
    p->centroid = center;
    Xf xf; xf.p = center; xf.q = rot(angle);
    for (int i = 0; i < 4; ++i) {
        p->v[i] = mul_xv(xf, p->v[i]);
        p->n[i] = mul_rv(xf.q, p->n[i]);
    }
}

void b2o_poly_set(Poly* p, const V2* vertices, int count) {
    p->radius = POLY_RADIUS;
    int n = count < B2_MAX_POLY ? count : B2_MAX_POLY;
    V2 ps[B2_MAX_POLY];
    int tempCount = 0;
    for (int i = 0; i < n; ++i) {
        V2 v = vertices[i];
        int unique = 1;
        for (int j = 0; j < tempCount; ++j) {
            V2 d = vsub(v, ps[j]);
            if (vlensq(d) < ((0.5f * LINEAR_SLOP) * (0.5f * LINEAR_SLOP))) { unique = 0; break; }
        }
        if (unique) ps[tempCount++] = v;
    }
    n = tempCount;
    /* gift wrapping, starting at the right-most (then lowest) point */
    int i0 = 0; float x0 = ps[0].x;
    for (int i = 1; i < n; ++i) {
        float x = ps[i].x;
        if (x > x0 || (x == x0 && ps[i].y < ps[i0].y)) { i0 = i; x0 = x; }
    }
    int hull[B2_MAX_POLY]; int m = 0; int ih = i0;
    for (;;) {
        hull[m] = ih;
        int ie = 0;
        for (int j = 1; j < n; ++j) {
            if (ie == ih) { ie = j; continue; }
            V2 r = vsub(ps[ie], ps[hull[m]]);
            V2 v = vsub(ps[j], ps[hull[m]]);
            float c = vcross(r, v);
            if (c < 0.0f) ie = j;
            if (c == 0.0f && vlensq(v) > vlensq(r)) ie = j;
        }
        ++m; ih = ie;
        if (ie == i0) break;
    }
    p->count = m;
    for (int i = 0; i < m; ++i) p->v[i] = ps[hull[i]];
    for (int i = 0; i < m; ++i) {
        int i2 = i + 1 < m ? i + 1 : 0;
        V2 edge = vsub(p->v[i2], p->v[i]);
        p->n[i] = vcross_vs(edge, 1.0f);
        vnormalize(&p->n[i]);
    }
    p->centroid = compute_centroid(p->v, m);
}

void b2o_poly_mass(const Poly* p, float density, float* mass, V2* center_out, float* I_out) {
    V2 center = v2(0.0f, 0.0f);
    float area = 0.0f, I = 0.0f;
    V2 s = v2(0.0f, 0.0f);
    for (int i = 0; i < p->count; ++i) s = vadd(s, p->v[i]);
    { float inv = 1.0f / p->count; s.x *= inv; s.y *= inv; }
    const float k_inv3 = 1.0f / 3.0f;
    for (int i = 0; i < p->count; ++i) {
        V2 e1 = vsub(p->v[i], s);
        V2 e2 = i + 1 < p->count ? vsub(p->v[i + 1], s) : vsub(p->v[0], s);
        float D = vcross(e1, e2);
        float triangleArea = 0.5f * D;
        area += triangleArea;
        center = vadd(center, vmul(triangleArea * k_inv3, vadd(e1, e2)));
        float ex1 = e1.x, ey1 = e1.y, ex2 = e2.x, ey2 = e2.y;
        float intx2 = ex1 * ex1 + ex2 * ex1 + ex2 * ex2;
        float inty2 = ey1 * ey1 + ey2 * ey1 + ey2 * ey2;
        I += (0.25f * k_inv3 * D) * (intx2 + inty2);
    }
    float m = density * area;
    { float inv = 1.0f / area; center.x *= inv; center.y *= inv; }
    V2 c = vadd(center, s);
    float Id = density * I;
    Id += m * (vdot(c, c) - vdot(center, center));
    *mass = m; *center_out = c; *I_out = Id;
}

static void poly_aabb(const Poly* p, Xf xf, AABB* out) {
    V2 lower = mul_xv(xf, p->v[0]);
    V2 upper = lower;
    for (int i = 1; i < p->count; ++i) {
        V2 v = mul_xv(xf, p->v[i]);
        lower = vmin(lower, v); upper = vmax(upper, v);
    }
    V2 r = v2(p->radius, p->radius);
    out->lo = vsub(lower, r); out->hi = vadd(upper, r);
}

/* ---------------------------------------------------------------- dynamic tree [B2 b2DynamicTree.cpp] */
static void tree_init(Tree* t) {
    t->root = NULLN;
    t->nodeCapacity = 16; t->nodeCount = 0;
    t->nodes = (TreeNode*)calloc((size_t)t->nodeCapacity, sizeof(TreeNode));
    for (int i = 0; i < t->nodeCapacity - 1; ++i) { t->nodes[i].parent = i + 1; t->nodes[i].height = -1; }
    t->nodes[t->nodeCapacity - 1].parent = NULLN; t->nodes[t->nodeCapacity - 1].height = -1;
    t->freeList = 0; t->insertionCount = 0; t->maxId = -1;
}
static int tree_alloc(Tree* t) {
    if (t->freeList == NULLN) {
        TreeNode* old = t->nodes;
        t->nodeCapacity *= 2;
        t->nodes = (TreeNode*)calloc((size_t)t->nodeCapacity, sizeof(TreeNode));
        memcpy(t->nodes, old, (size_t)t->nodeCount * sizeof(TreeNode));
        free(old);
        for (int i = t->nodeCount; i < t->nodeCapacity - 1; ++i) { t->nodes[i].parent = i + 1; t->nodes[i].height = -1; }
        t->nodes[t->nodeCapacity - 1].parent = NULLN; t->nodes[t->nodeCapacity - 1].height = -1;
        t->freeList = t->nodeCount;
    }
    int id = t->freeList;
    t->freeList = t->nodes[id].parent;
    t->nodes[id].parent = NULLN; t->nodes[id].child1 = NULLN; t->nodes[id].child2 = NULLN;
    t->nodes[id].height = 0; t->nodes[id].userData = NULL;
    ++t->nodeCount;
    if (id > t->maxId) t->maxId = id;
    return id;
}
static void tree_free(Tree* t, int id) {
    t->nodes[id].parent = t->freeList; t->nodes[id].height = -1; t->freeList = id; --t->nodeCount;
}
static inline int is_leaf(const TreeNode* n) { return n->child1 == NULLN; }

static int tree_balance(Tree* t, int iA) {
    TreeNode* A = t->nodes + iA;
    if (is_leaf(A) || A->height < 2) return iA;
    int iB = A->child1, iC = A->child2;
    TreeNode* B = t->nodes + iB; TreeNode* C = t->nodes + iC;
    int balance = C->height - B->height;
    if (balance > 1) {
        int iF = C->child1, iG = C->child2;
        TreeNode* F = t->nodes + iF; TreeNode* G = t->nodes + iG;
        C->child1 = iA; C->parent = A->parent; A->parent = iC;
        if (C->parent != NULLN) {
            if (t->nodes[C->parent].child1 == iA) t->nodes[C->parent].child1 = iC;
            else t->nodes[C->parent].child2 = iC;
        } else t->root = iC;
        if (F->height > G->height) {
            C->child2 = iF; A->child2 = iG; G->parent = iA;
            A->aabb = aabb_combine(B->aabb, G->aabb); C->aabb = aabb_combine(A->aabb, F->aabb);
            A->height = 1 + (B->height > G->height ? B->height : G->height);
            C->height = 1 + (A->height > F->height ? A->height : F->height);
        } else {
            C->child2 = iG; A->child2 = iF; F->parent = iA;
            A->aabb = aabb_combine(B->aabb, F->aabb); C->aabb = aabb_combine(A->aabb, G->aabb);
            A->height = 1 + (B->height > F->height ? B->height : F->height);
            C->height = 1 + (A->height > G->height ? A->height : G->height);
        }
        return iC;
    }
    if (balance < -1) {
        int iD = B->child1, iE = B->child2;
        TreeNode* D = t->nodes + iD; TreeNode* E = t->nodes + iE;
        B->child1 = iA; B->parent = A->parent; A->parent = iB;
        if (B->parent != NULLN) {
            if (t->nodes[B->parent].child1 == iA) t->nodes[B->parent].child1 = iB;
            else t->nodes[B->parent].child2 = iB;
        } else t->root = iB;
        if (D->height > E->height) {
            B->child2 = iD; A->child1 = iE; E->parent = iA;
            A->aabb = aabb_combine(C->aabb, E->aabb); B->aabb = aabb_combine(A->aabb, D->aabb);
            A->height = 1 + (C->height > E->height ? C->height : E->height);
            B->height = 1 + (A->height > D->height ? A->height : D->height);
        } else {
            B->child2 = iE; A->child1 = iD; D->parent = iA;
            A->aabb = aabb_combine(C->aabb, D->aabb); B->aabb = aabb_combine(A->aabb, E->aabb);
            A->height = 1 + (C->height > D->height ? C->height : D->height);
            B->height = 1 + (A->height > E->height ? A->height : E->height);
        }
        return iB;
    }
    return iA;
}

static void tree_insert_leaf(Tree* t, int leaf) {
    ++t->insertionCount;
    if (t->root == NULLN) { t->root = leaf; t->nodes[leaf].parent = NULLN; return; }
    AABB leafAABB = t->nodes[leaf].aabb;
    int index = t->root;
    while (!is_leaf(t->nodes + index)) {
        int child1 = t->nodes[index].child1, child2 = t->nodes[index].child2;
        float area = aabb_perimeter(t->nodes[index].aabb);
        AABB combined = aabb_combine(t->nodes[index].aabb, leafAABB);
        float combinedArea = aabb_perimeter(combined);
        float cost = 2.0f * combinedArea;
        float inheritanceCost = 2.0f * (combinedArea - area);
        float cost1, cost2;
        if (is_leaf(t->nodes + child1)) {
            AABB a = aabb_combine(leafAABB, t->nodes[child1].aabb);
            cost1 = aabb_perimeter(a) + inheritanceCost;
        } else {
            AABB a = aabb_combine(leafAABB, t->nodes[child1].aabb);
            float oldArea = aabb_perimeter(t->nodes[child1].aabb);
            float newArea = aabb_perimeter(a);
            cost1 = (newArea - oldArea) + inheritanceCost;
        }
        if (is_leaf(t->nodes + child2)) {
            AABB a = aabb_combine(leafAABB, t->nodes[child2].aabb);
            cost2 = aabb_perimeter(a) + inheritanceCost;
        } else {
            AABB a = aabb_combine(leafAABB, t->nodes[child2].aabb);
            float oldArea = aabb_perimeter(t->nodes[child2].aabb);
            float newArea = aabb_perimeter(a);
            cost2 = newArea - oldArea + inheritanceCost;
        }
        if (cost < cost1 && cost < cost2) break;
        index = cost1 < cost2 ? child1 : child2;
    }
    int sibling = index;
    int oldParent = t->nodes[sibling].parent;
    int newParent = tree_alloc(t);
    t->nodes[newParent].parent = oldParent;
    t->nodes[newParent].userData = NULL;
    t->nodes[newParent].aabb = aabb_combine(leafAABB, t->nodes[sibling].aabb);
    t->nodes[newParent].height = t->nodes[sibling].height + 1;
    if (oldParent != NULLN) {
        if (t->nodes[oldParent].child1 == sibling) t->nodes[oldParent].child1 = newParent;
        else t->nodes[oldParent].child2 = newParent;
    } else {
        t->root = newParent;
    }
    t->nodes[newParent].child1 = sibling; t->nodes[newParent].child2 = leaf;
    t->nodes[sibling].parent = newParent; t->nodes[leaf].parent = newParent;
    index = t->nodes[leaf].parent;
    while (index != NULLN) {
        index = tree_balance(t, index);
        int c1 = t->nodes[index].child1, c2 = t->nodes[index].child2;
        int h1 = t->nodes[c1].height, h2 = t->nodes[c2].height;
        t->nodes[index].height = 1 + (h1 > h2 ? h1 : h2);
        t->nodes[index].aabb = aabb_combine(t->nodes[c1].aabb, t->nodes[c2].aabb);
        index = t->nodes[index].parent;
    }
}

static void tree_remove_leaf(Tree* t, int leaf) {
    if (leaf == t->root) { t->root = NULLN; return; }
    int parent = t->nodes[leaf].parent;
    int grandParent = t->nodes[parent].parent;
    int sibling = t->nodes[parent].child1 == leaf ? t->nodes[parent].child2 : t->nodes[parent].child1;
    if (grandParent != NULLN) {
        if (t->nodes[grandParent].child1 == parent) t->nodes[grandParent].child1 = sibling;
        else t->nodes[grandParent].child2 = sibling;
        t->nodes[sibling].parent = grandParent;
        tree_free(t, parent);
        int index = grandParent;
        while (index != NULLN) {
            index = tree_balance(t, index);
            int c1 = t->nodes[index].child1, c2 = t->nodes[index].child2;
            t->nodes[index].aabb = aabb_combine(t->nodes[c1].aabb, t->nodes[c2].aabb);
            int h1 = t->nodes[c1].height, h2 = t->nodes[c2].height;
            t->nodes[index].height = 1 + (h1 > h2 ? h1 : h2);
            index = t->nodes[index].parent;
        }
    } else {
        t->root = sibling;
        t->nodes[sibling].parent = NULLN;
        tree_free(t, parent);
    }
}

static int tree_create_proxy(Tree* t, AABB aabb, void* userData) {
    int id = tree_alloc(t);
    V2 r = v2(AABB_EXT, AABB_EXT);
    t->nodes[id].aabb.lo = vsub(aabb.lo, r);
    t->nodes[id].aabb.hi = vadd(aabb.hi, r);
    t->nodes[id].userData = userData;
    t->nodes[id].height = 0;
    tree_insert_leaf(t, id);
    return id;
}
static void tree_destroy_proxy(Tree* t, int id) { tree_remove_leaf(t, id); tree_free(t, id); }
static int tree_move_proxy(Tree* t, int id, AABB aabb, V2 displacement) {
    if (aabb_contains(t->nodes[id].aabb, aabb)) return 0;
    tree_remove_leaf(t, id);
    AABB b = aabb;
    V2 r = v2(AABB_EXT, AABB_EXT);
    b.lo = vsub(b.lo, r); b.hi = vadd(b.hi, r);
    V2 d = vmul(AABB_MUL, displacement);
    if (d.x < 0.0f) b.lo.x += d.x; else b.hi.x += d.x;
    if (d.y < 0.0f) b.lo.y += d.y; else b.hi.y += d.y;
    t->nodes[id].aabb = b;
    tree_insert_leaf(t, id);
    return 1;
}

/* ---------------------------------------------------------------- broad phase [B2 b2BroadPhase.cpp] */
static void bp_init(BroadPhase* bp) {
    tree_init(&bp->tree); bp->proxyCount = 0;
    bp->moveCap = 16; bp->moveCount = 0; bp->moveBuf = (int*)malloc(sizeof(int) * (size_t)bp->moveCap);
    bp->pairCap = 16; bp->pairCount = 0; bp->pairBuf = (Pair*)malloc(sizeof(Pair) * (size_t)bp->pairCap);
}
static void bp_buffer_move(BroadPhase* bp, int id) {
    if (bp->moveCount == bp->moveCap) { bp->moveCap *= 2; bp->moveBuf = (int*)realloc(bp->moveBuf, sizeof(int) * (size_t)bp->moveCap); }
    bp->moveBuf[bp->moveCount++] = id;
    if (bp->moveCount > bp->maxMove) bp->maxMove = bp->moveCount;
}
static void bp_unbuffer_move(BroadPhase* bp, int id) {
    for (int i = 0; i < bp->moveCount; ++i) if (bp->moveBuf[i] == id) bp->moveBuf[i] = NULLN;
}
static int bp_create_proxy(BroadPhase* bp, AABB aabb, void* ud) {
    int id = tree_create_proxy(&bp->tree, aabb, ud); ++bp->proxyCount; bp_buffer_move(bp, id); return id;
}
static void bp_destroy_proxy(BroadPhase* bp, int id) { bp_unbuffer_move(bp, id); --bp->proxyCount; tree_destroy_proxy(&bp->tree, id); }
static void bp_move_proxy(BroadPhase* bp, int id, AABB aabb, V2 disp) {
    if (tree_move_proxy(&bp->tree, id, aabb, disp)) bp_buffer_move(bp, id);
}
static int pair_cmp(const void* a, const void* b) {
    const Pair* p = (const Pair*)a; const Pair* q = (const Pair*)b;
    if (p->a != q->a) return p->a < q->a ? -1 : 1;
    if (p->b != q->b) return p->b < q->b ? -1 : 1;
    return 0;
}
static void bp_query_cb(BroadPhase* bp, int proxyId) {
    if (proxyId == bp->queryProxyId) return;
    if (bp->pairCount == bp->pairCap) { bp->pairCap *= 2; bp->pairBuf = (Pair*)realloc(bp->pairBuf, sizeof(Pair) * (size_t)bp->pairCap); }
    int q = bp->queryProxyId;
    bp->pairBuf[bp->pairCount].a = proxyId < q ? proxyId : q;
    bp->pairBuf[bp->pairCount].b = proxyId > q ? proxyId : q;
    ++bp->pairCount;
}
static void tree_query(BroadPhase* bp, AABB aabb) {
    Tree* t = &bp->tree;
    int stack[256]; int n = 0;
    stack[n++] = t->root;
    while (n > 0) {
        int id = stack[--n];
        if (id == NULLN) continue;
        const TreeNode* node = t->nodes + id;
        if (aabb_overlap(node->aabb, aabb)) {
            if (is_leaf(node)) bp_query_cb(bp, id);
            else { stack[n++] = node->child1; stack[n++] = node->child2; }
        }
    }
}

/* ---------------------------------------------------------------- narrow phase [B2 b2CollidePolygon.cpp] */
typedef struct { V2 v; uint32_t id; } ClipVertex;
static inline uint32_t cf_make(int indexA, int indexB, int typeA, int typeB) {
    return (uint32_t)(uint8_t)indexA | ((uint32_t)(uint8_t)indexB << 8) | ((uint32_t)(uint8_t)typeA << 16) | ((uint32_t)(uint8_t)typeB << 24);
}
#define CF_VERTEX 0
#define CF_FACE 1

static float find_max_separation(int* edgeIndex, const Poly* poly1, Xf xf1, const Poly* poly2, Xf xf2) {
    int count1 = poly1->count, count2 = poly2->count;
    Xf xf = mulT_xx(xf2, xf1);
    int bestIndex = 0; float maxSeparation = -FLT_MAX;
    for (int i = 0; i < count1; ++i) {
        V2 n = mul_rv(xf.q, poly1->n[i]);
        V2 v1 = mul_xv(xf, poly1->v[i]);
        float si = FLT_MAX;
        for (int j = 0; j < count2; ++j) {
            float sij = vdot(n, vsub(poly2->v[j], v1));
            if (sij < si) si = sij;
        }
        if (si > maxSeparation) { maxSeparation = si; bestIndex = i; }
    }
    *edgeIndex = bestIndex;
    return maxSeparation;
}

static void find_incident_edge(ClipVertex c[2], const Poly* poly1, Xf xf1, int edge1, const Poly* poly2, Xf xf2) {
    int count2 = poly2->count;
    V2 normal1 = mulT_rv(xf2.q, mul_rv(xf1.q, poly1->n[edge1]));
    int index = 0; float minDot = FLT_MAX;
    for (int i = 0; i < count2; ++i) {
        float d = vdot(normal1, poly2->n[i]);
        if (d < minDot) { minDot = d; index = i; }
    }
    int i1 = index, i2 = i1 + 1 < count2 ? i1 + 1 : 0;
    c[0].v = mul_xv(xf2, poly2->v[i1]); c[0].id = cf_make(edge1, i1, CF_FACE, CF_VERTEX);
    c[1].v = mul_xv(xf2, poly2->v[i2]); c[1].id = cf_make(edge1, i2, CF_FACE, CF_VERTEX);
}

static int clip_segment_to_line(ClipVertex vOut[2], const ClipVertex vIn[2], V2 normal, float offset, int vertexIndexA) {
    int numOut = 0;
    float distance0 = vdot(normal, vIn[0].v) - offset;
    float distance1 = vdot(normal, vIn[1].v) - offset;
    if (distance0 <= 0.0f) vOut[numOut++] = vIn[0];
    if (distance1 <= 0.0f) vOut[numOut++] = vIn[1];
    if (distance0 * distance1 < 0.0f) {
        float interp = distance0 / (distance0 - distance1);
        vOut[numOut].v = vadd(vIn[0].v, vmul(interp, vsub(vIn[1].v, vIn[0].v)));
        vOut[numOut].id = cf_make(vertexIndexA, (int)((vIn[0].id >> 8) & 0xff), CF_VERTEX, CF_FACE);
        ++numOut;
    }
    return numOut;
}

static void collide_polygons(Manifold* manifold, const Poly* polyA, Xf xfA, const Poly* polyB, Xf xfB) {
    manifold->pointCount = 0;
    float totalRadius = polyA->radius + polyB->radius;
    int edgeA = 0;
    float separationA = find_max_separation(&edgeA, polyA, xfA, polyB, xfB);
    if (separationA > totalRadius) return;
    int edgeB = 0;
    float separationB = find_max_separation(&edgeB, polyB, xfB, polyA, xfA);
    if (separationB > totalRadius) return;
    const Poly *poly1, *poly2; Xf xf1, xf2; int edge1; int flip;
    const float k_tol = 0.1f * LINEAR_SLOP;
    if (separationB > separationA + k_tol) {
        poly1 = polyB; poly2 = polyA; xf1 = xfB; xf2 = xfA; edge1 = edgeB; manifold->type = MT_FACEB; flip = 1;
    } else {
        poly1 = polyA; poly2 = polyB; xf1 = xfA; xf2 = xfB; edge1 = edgeA; manifold->type = MT_FACEA; flip = 0;
    }
    ClipVertex incidentEdge[2];
    find_incident_edge(incidentEdge, poly1, xf1, edge1, poly2, xf2);
    int count1 = poly1->count;
    int iv1 = edge1, iv2 = edge1 + 1 < count1 ? edge1 + 1 : 0;
    V2 v11 = poly1->v[iv1], v12 = poly1->v[iv2];
    V2 localTangent = vsub(v12, v11);
    vnormalize(&localTangent);
    V2 localNormal = vcross_vs(localTangent, 1.0f);
    V2 planePoint = vmul(0.5f, vadd(v11, v12));
    V2 tangent = mul_rv(xf1.q, localTangent);
    V2 normal = vcross_vs(tangent, 1.0f);
    v11 = mul_xv(xf1, v11); v12 = mul_xv(xf1, v12);
    float frontOffset = vdot(normal, v11);
    float sideOffset1 = -vdot(tangent, v11) + totalRadius;
    float sideOffset2 = vdot(tangent, v12) + totalRadius;
    ClipVertex cp1[2], cp2[2];
    int np = clip_segment_to_line(cp1, incidentEdge, vneg(tangent), sideOffset1, iv1);
    if (np < 2) return;
    np = clip_segment_to_line(cp2, cp1, tangent, sideOffset2, iv2);
    if (np < 2) return;
    manifold->localNormal = localNormal;
    manifold->localPoint = planePoint;
    int pointCount = 0;
    for (int i = 0; i < 2; ++i) {
        float separation = vdot(normal, cp2[i].v) - frontOffset;
        if (separation <= totalRadius) {
            MPoint* cp = manifold->points + pointCount;
            cp->localPoint = mulT_xv(xf2, cp2[i].v);
            uint32_t id = cp2[i].id;
            if (flip) {
                uint32_t iA = id & 0xff, iB = (id >> 8) & 0xff, tA = (id >> 16) & 0xff, tB = (id >> 24) & 0xff;
                id = iB | (iA << 8) | (tB << 16) | (tA << 24);
            }
            cp->id = id;
            ++pointCount;
        }
    }
    manifold->pointCount = pointCount;
}

/* ---------------------------------------------------------------- contacts [B2 b2Contact.cpp, b2ContactManager.cpp] */
static Contact* contact_create(Fixture* fA, Fixture* fB) {
    Contact* c = (Contact*)calloc(1, sizeof(Contact));
    c->flags = CF_ENABLED;
    c->fA = fA; c->fB = fB;
    c->manifold.pointCount = 0;
    c->toiCount = 0;
    c->friction = sqrtf(fA->friction * fB->friction);
    c->restitution = fA->restitution > fB->restitution ? fA->restitution : fB->restitution;
    c->tangentSpeed = 0.0f;
    return c;
}

static void contact_update(Contact* c, ContactManager* cm) {
    Manifold oldManifold = c->manifold;
    c->flags |= CF_ENABLED;
    int wasTouching = (c->flags & CF_TOUCHING) == CF_TOUCHING;
    Body* bA = c->fA->body; Body* bB = c->fB->body;
    collide_polygons(&c->manifold, &c->fA->shape, bA->xf, &c->fB->shape, bB->xf);
    cm->satCalls++;
    int touching = c->manifold.pointCount > 0;
    for (int i = 0; i < c->manifold.pointCount; ++i) {
        MPoint* mp2 = c->manifold.points + i;
        mp2->normalImpulse = 0.0f; mp2->tangentImpulse = 0.0f;
        for (int j = 0; j < oldManifold.pointCount; ++j) {
            MPoint* mp1 = oldManifold.points + j;
            if (mp1->id == mp2->id) { mp2->normalImpulse = mp1->normalImpulse; mp2->tangentImpulse = mp1->tangentImpulse; break; }
        }
    }
    if (touching) c->flags |= CF_TOUCHING; else c->flags &= ~CF_TOUCHING;
    if (!wasTouching && touching && cm->begin) cm->begin(cm->listenerCtx, c);
    if (wasTouching && !touching && cm->end) cm->end(cm->listenerCtx, c);
}

static void cm_destroy(ContactManager* cm, Contact* c) {
    Body* bA = c->fA->body; Body* bB = c->fB->body;
    if (cm->end && (c->flags & CF_TOUCHING)) cm->end(cm->listenerCtx, c);
    if (c->prev) c->prev->next = c->next;
    if (c->next) c->next->prev = c->prev;
    if (c == cm->contactList) cm->contactList = c->next;
    if (c->nodeA.prev) c->nodeA.prev->next = c->nodeA.next;
    if (c->nodeA.next) c->nodeA.next->prev = c->nodeA.prev;
    if (&c->nodeA == bA->contactList) bA->contactList = c->nodeA.next;
    if (c->nodeB.prev) c->nodeB.prev->next = c->nodeB.next;
    if (c->nodeB.next) c->nodeB.next->prev = c->nodeB.prev;
    if (&c->nodeB == bB->contactList) bB->contactList = c->nodeB.next;
    free(c);
    --cm->contactCount;
}

static int body_should_collide(const Body* a, const Body* b) {
    if (a->type != BT_DYNAMIC && b->type != BT_DYNAMIC) return 0;
    return 1;
}

static void cm_add_pair(ContactManager* cm, Fixture* fixtureA, Fixture* fixtureB) {
    Body* bodyA = fixtureA->body; Body* bodyB = fixtureB->body;
    if (bodyA == bodyB) return;
    for (ContactEdge* e = bodyB->contactList; e; e = e->next) {
        if (e->other == bodyA) {
            Fixture* fA = e->contact->fA; Fixture* fB = e->contact->fB;
            if (fA == fixtureA && fB == fixtureB) return;
            if (fA == fixtureB && fB == fixtureA) return;
        }
    }
    if (!body_should_collide(bodyB, bodyA)) return;
    Contact* c = contact_create(fixtureA, fixtureB);
    c->prev = NULL; c->next = cm->contactList;
    if (cm->contactList) cm->contactList->prev = c;
    cm->contactList = c;
    c->nodeA.contact = c; c->nodeA.other = bodyB; c->nodeA.prev = NULL; c->nodeA.next = bodyA->contactList;
    if (bodyA->contactList) bodyA->contactList->prev = &c->nodeA;
    bodyA->contactList = &c->nodeA;
    c->nodeB.contact = c; c->nodeB.other = bodyA; c->nodeB.prev = NULL; c->nodeB.next = bodyB->contactList;
    if (bodyB->contactList) bodyB->contactList->prev = &c->nodeB;
    bodyB->contactList = &c->nodeB;
    bodyA->flags |= BF_AWAKE; bodyB->flags |= BF_AWAKE;
    ++cm->contactCount;
    if (cm->contactCount > cm->maxContacts) cm->maxContacts = cm->contactCount;
}

static void cm_find_new_contacts(ContactManager* cm) {
    BroadPhase* bp = &cm->bp;
    bp->pairCount = 0;
    for (int i = 0; i < bp->moveCount; ++i) {
        bp->queryProxyId = bp->moveBuf[i];
        if (bp->queryProxyId == NULLN) continue;
        tree_query(bp, bp->tree.nodes[bp->queryProxyId].aabb);
    }
    bp->moveCount = 0;
    qsort(bp->pairBuf, (size_t)bp->pairCount, sizeof(Pair), pair_cmp);
    int i = 0;
    while (i < bp->pairCount) {
        Pair* primary = bp->pairBuf + i;
        Fixture* fA = (Fixture*)bp->tree.nodes[primary->a].userData;
        Fixture* fB = (Fixture*)bp->tree.nodes[primary->b].userData;
        cm_add_pair(cm, fA, fB);
        ++i;
        while (i < bp->pairCount) {
            Pair* p = bp->pairBuf + i;
            if (p->a != primary->a || p->b != primary->b) break;
            ++i;
        }
    }
}

static void cm_collide(ContactManager* cm) {
    Contact* c = cm->contactList;
    while (c) {
        Body* bA = c->fA->body; Body* bB = c->fB->body;
        int activeA = (bA->flags & BF_AWAKE) && bA->type != BT_STATIC;
        int activeB = (bB->flags & BF_AWAKE) && bB->type != BT_STATIC;
        if (!activeA && !activeB) { c = c->next; continue; }
        int overlap = aabb_overlap(cm->bp.tree.nodes[c->fA->proxyId].aabb, cm->bp.tree.nodes[c->fB->proxyId].aabb);
        if (!overlap) { Contact* nuke = c; c = nuke->next; cm_destroy(cm, nuke); continue; }
        contact_update(c, cm);
        c = c->next;
    }
}

/* ---------------------------------------------------------------- bodies / fixtures [B2 b2Body.cpp, b2Fixture.cpp] */
static void body_synchronize_transform(Body* b) {
    b->xf.q = rot(b->sweep.a);
    b->xf.p = vsub(b->sweep.c, mul_rv(b->xf.q, b->sweep.localCenter));
}

static void body_reset_mass(Body* b) {
    b->mass = 0.0f; b->invMass = 0.0f; b->I = 0.0f; b->invI = 0.0f;
    b->sweep.localCenter = v2(0.0f, 0.0f);
    if (b->type == BT_STATIC || b->type == BT_KINEMATIC) {
        b->sweep.c0 = b->xf.p; b->sweep.c = b->xf.p; b->sweep.a0 = b->sweep.a;
        return;
    }
    V2 localCenter = v2(0.0f, 0.0f);
    for (Fixture* f = b->fixtureList; f; f = f->next) {
        if (f->density == 0.0f) continue;
        float m; V2 c; float I;
        b2o_poly_mass(&f->shape, f->density, &m, &c, &I);
        b->mass += m;
        localCenter = vadd(localCenter, vmul(m, c));
        b->I += I;
    }
    if (b->mass > 0.0f) {
        b->invMass = 1.0f / b->mass;
        localCenter.x *= b->invMass; localCenter.y *= b->invMass;
    } else {
        b->mass = 1.0f; b->invMass = 1.0f;
    }
    if (b->I > 0.0f && (b->flags & BF_FIXEDROT) == 0) {
        b->I -= b->mass * vdot(localCenter, localCenter);
        b->invI = 1.0f / b->I;
    } else {
        b->I = 0.0f; b->invI = 0.0f;
    }
    V2 oldCenter = b->sweep.c;
    b->sweep.localCenter = localCenter;
    b->sweep.c0 = b->sweep.c = mul_xv(b->xf, b->sweep.localCenter);
    b->v = vadd(b->v, vcross_sv(b->w, vsub(b->sweep.c, oldCenter)));
}

static void body_synchronize_fixtures(Body* b) {
    Xf xf1;
    xf1.q = rot(b->sweep.a0);
    xf1.p = vsub(b->sweep.c0, mul_rv(xf1.q, b->sweep.localCenter));
    BroadPhase* bp = &b->world->cm.bp;
    for (Fixture* f = b->fixtureList; f; f = f->next) {
        AABB a1, a2;
        poly_aabb(&f->shape, xf1, &a1);
        poly_aabb(&f->shape, b->xf, &a2);
        f->aabb = aabb_combine(a1, a2);
        V2 disp = vsub(b->xf.p, xf1.p);
        bp_move_proxy(bp, f->proxyId, f->aabb, disp);
    }
}

static void body_advance(Body* b, float alpha) {
    sweep_advance(&b->sweep, alpha);
    b->sweep.c = b->sweep.c0;
    b->sweep.a = b->sweep.a0;
    b->xf.q = rot(b->sweep.a);
    b->xf.p = vsub(b->sweep.c, mul_rv(b->xf.q, b->sweep.localCenter));
}

World* b2o_world_create(void) {
    World* w = (World*)calloc(1, sizeof(World));
    bp_init(&w->cm.bp);
    w->cm.contactList = NULL; w->cm.contactCount = 0;
    w->inv_dt0 = 0.0f;
    w->flags = WF_CLEARFORCES;
    w->stepComplete = 1;
    w->gravity = v2(0.0f, 0.0f);
    return w;
}

void b2o_set_listener(World* w, ContactCb begin, ContactCb end, void* ctx) {
    w->cm.begin = begin; w->cm.end = end; w->cm.listenerCtx = ctx;
}

Body* b2o_create_body(World* w, const BodyDef* def) {
    Body* b = (Body*)calloc(1, sizeof(Body));
    b->flags = BF_AWAKE | BF_AUTOSLEEP | BF_ACTIVE;
    b->world = w;
    b->xf.p = def->position;
    b->xf.q = rot(def->angle);
    b->sweep.localCenter = v2(0.0f, 0.0f);
    b->sweep.c0 = b->xf.p; b->sweep.c = b->xf.p;
    b->sweep.a0 = def->angle; b->sweep.a = def->angle; b->sweep.alpha0 = 0.0f;
    b->linearDamping = def->linearDamping; b->angularDamping = def->angularDamping;
    b->gravityScale = 1.0f;
    b->type = def->type;
    if (b->type == BT_DYNAMIC) { b->mass = 1.0f; b->invMass = 1.0f; } else { b->mass = 0.0f; b->invMass = 0.0f; }
    b->I = 0.0f; b->invI = 0.0f;
    b->tag = def->tag;
    b->prev = NULL; b->next = w->bodyList;
    if (w->bodyList) w->bodyList->prev = b;
    w->bodyList = b;
    ++w->bodyCount;
    return b;
}

Fixture* b2o_create_fixture(Body* b, const FixtureDef* def) {
    Fixture* f = (Fixture*)calloc(1, sizeof(Fixture));
    f->shape = *def->shape;
    f->density = def->density; f->friction = def->friction; f->restitution = def->restitution;
    f->tag = def->tag;
    f->body = b;
    /* CreateProxies with the body's current transform */
    poly_aabb(&f->shape, b->xf, &f->aabb);
    f->proxyId = bp_create_proxy(&b->world->cm.bp, f->aabb, f);
    f->next = b->fixtureList; b->fixtureList = f; ++b->fixtureCount;
    if (f->density > 0.0f) body_reset_mass(b);
    b->world->flags |= WF_NEWFIXTURE;
    return f;
}

void b2o_destroy_body(World* w, Body* b) {
    ContactEdge* ce = b->contactList;
    while (ce) { ContactEdge* ce0 = ce; ce = ce->next; cm_destroy(&w->cm, ce0->contact); }
    b->contactList = NULL;
    Fixture* f = b->fixtureList;
    while (f) {
        Fixture* f0 = f; f = f->next;
        bp_destroy_proxy(&w->cm.bp, f0->proxyId);
        free(f0);
        b->fixtureList = f; b->fixtureCount -= 1;
    }
    if (b->prev) b->prev->next = b->next;
    if (b->next) b->next->prev = b->prev;
    if (b == w->bodyList) w->bodyList = b->next;
    --w->bodyCount;
    free(b);
}

void b2o_world_destroy(World* w) {
    Body* b = w->bodyList;
    while (b) { Body* n = b->next; b2o_destroy_body(w, b); b = n; }
    free(w->cm.bp.tree.nodes); free(w->cm.bp.moveBuf); free(w->cm.bp.pairBuf);
    free(w);
}

/* body API (pybox2d property setters / Apply* methods) [B2 b2Body.h] */
void b2o_set_linear_velocity(Body* b, V2 v) {
    if (b->type == BT_STATIC) return;
    if (vdot(v, v) > 0.0f) b->flags |= BF_AWAKE;
    b->v = v;
}
void b2o_set_angular_velocity(Body* b, float w) {
    if (b->type == BT_STATIC) return;
    if (w * w > 0.0f) b->flags |= BF_AWAKE;
    b->w = w;
}
void b2o_apply_force(Body* b, V2 force, V2 point) {
    if (b->type != BT_DYNAMIC) return;
    b->force = vadd(b->force, force);
    b->torque += vcross(vsub(point, b->sweep.c), force);
}
void b2o_apply_linear_impulse(Body* b, V2 impulse, V2 point) {
    if (b->type != BT_DYNAMIC) return;
    b->v = vadd(b->v, vmul(b->invMass, impulse));
    b->w += b->invI * vcross(vsub(point, b->sweep.c), impulse);
}
void b2o_apply_angular_impulse(Body* b, float impulse) { if (b->type != BT_DYNAMIC) return; b->w += b->invI * impulse; }
void b2o_apply_torque(Body* b, float torque) { if (b->type != BT_DYNAMIC) return; b->torque += torque; }
V2 b2o_world_point(const Body* b, V2 local) { return mul_xv(b->xf, local); }
V2 b2o_world_vector(const Body* b, V2 local) { return mul_rv(b->xf.q, local); }
float b2o_inertia(const Body* b) { return b->I + b->mass * vdot(b->sweep.localCenter, b->sweep.localCenter); }

/* ---------------------------------------------------------------- contact solver [B2 b2ContactSolver.cpp] */
typedef struct { V2 c; float a; } Position;
typedef struct { V2 v; float w; } Velocity;
typedef struct { V2 rA, rB; float normalImpulse, tangentImpulse, normalMass, tangentMass, velocityBias; } VCPoint;
typedef struct {
    VCPoint points[2]; V2 normal; float nm[4]; /* normalMass ex.x ex.y ey.x ey.y */ float K[4];
    int indexA, indexB; float invMassA, invMassB, invIA, invIB, friction, restitution, tangentSpeed;
    int pointCount, contactIndex;
} VC;
typedef struct {
    V2 localPoints[2]; V2 localNormal, localPoint; int indexA, indexB; float invMassA, invMassB;
    V2 localCenterA, localCenterB; float invIA, invIB; int type; float radiusA, radiusB; int pointCount;
} PC;
typedef struct {
    float dt, inv_dt, dtRatio; int velocityIterations, positionIterations, warmStarting;
} TimeStep;
typedef struct {
    TimeStep step; Position* positions; Velocity* velocities; Contact** contacts; int count; VC* vcs; PC* pcs;
} Solver;

static void solver_init(Solver* s, TimeStep step, Contact** contacts, int count, Position* pos, Velocity* vel) {
    s->step = step; s->contacts = contacts; s->count = count; s->positions = pos; s->velocities = vel;
    s->vcs = (VC*)calloc((size_t)(count > 0 ? count : 1), sizeof(VC));
    s->pcs = (PC*)calloc((size_t)(count > 0 ? count : 1), sizeof(PC));
    for (int i = 0; i < count; ++i) {
        Contact* contact = contacts[i];
        Fixture* fA = contact->fA; Fixture* fB = contact->fB;
        float radiusA = fA->shape.radius, radiusB = fB->shape.radius;
        Body* bA = fA->body; Body* bB = fB->body;
        Manifold* manifold = &contact->manifold;
        int pointCount = manifold->pointCount;
        VC* vc = s->vcs + i;
        vc->friction = contact->friction; vc->restitution = contact->restitution; vc->tangentSpeed = contact->tangentSpeed;
        vc->indexA = bA->islandIndex; vc->indexB = bB->islandIndex;
        vc->invMassA = bA->invMass; vc->invMassB = bB->invMass; vc->invIA = bA->invI; vc->invIB = bB->invI;
        vc->contactIndex = i; vc->pointCount = pointCount;
        memset(vc->K, 0, sizeof(vc->K)); memset(vc->nm, 0, sizeof(vc->nm));
        PC* pc = s->pcs + i;
        pc->indexA = bA->islandIndex; pc->indexB = bB->islandIndex;
        pc->invMassA = bA->invMass; pc->invMassB = bB->invMass;
        pc->localCenterA = bA->sweep.localCenter; pc->localCenterB = bB->sweep.localCenter;
        pc->invIA = bA->invI; pc->invIB = bB->invI;
        pc->localNormal = manifold->localNormal; pc->localPoint = manifold->localPoint;
        pc->pointCount = pointCount; pc->radiusA = radiusA; pc->radiusB = radiusB; pc->type = manifold->type;
        for (int j = 0; j < pointCount; ++j) {
            MPoint* cp = manifold->points + j;
            VCPoint* vcp = vc->points + j;
            if (step.warmStarting) {
                vcp->normalImpulse = step.dtRatio * cp->normalImpulse;
                vcp->tangentImpulse = step.dtRatio * cp->tangentImpulse;
            } else {
                vcp->normalImpulse = 0.0f; vcp->tangentImpulse = 0.0f;
            }
            vcp->rA = v2(0.0f, 0.0f); vcp->rB = v2(0.0f, 0.0f);
            vcp->normalMass = 0.0f; vcp->tangentMass = 0.0f; vcp->velocityBias = 0.0f;
            pc->localPoints[j] = cp->localPoint;
        }
    }
}
static void solver_free(Solver* s) { free(s->vcs); free(s->pcs); }

static void world_manifold(const Manifold* m, Xf xfA, float radiusA, Xf xfB, float radiusB, V2* normal, V2 points[2]) {
    if (m->pointCount == 0) return;
    if (m->type == MT_FACEA) {
        *normal = mul_rv(xfA.q, m->localNormal);
        V2 planePoint = mul_xv(xfA, m->localPoint);
        for (int i = 0; i < m->pointCount; ++i) {
            V2 clipPoint = mul_xv(xfB, m->points[i].localPoint);
            V2 cA = vadd(clipPoint, vmul(radiusA - vdot(vsub(clipPoint, planePoint), *normal), *normal));
            V2 cB = vsub(clipPoint, vmul(radiusB, *normal));
            points[i] = vmul(0.5f, vadd(cA, cB));
        }
    } else {
        *normal = mul_rv(xfB.q, m->localNormal);
        V2 planePoint = mul_xv(xfB, m->localPoint);
        for (int i = 0; i < m->pointCount; ++i) {
            V2 clipPoint = mul_xv(xfA, m->points[i].localPoint);
            V2 cB = vadd(clipPoint, vmul(radiusB - vdot(vsub(clipPoint, planePoint), *normal), *normal));
            V2 cA = vsub(clipPoint, vmul(radiusA, *normal));
            points[i] = vmul(0.5f, vadd(cA, cB));
        }
        *normal = vneg(*normal);
    }
}

static void solver_init_velocity_constraints(Solver* s) {
    for (int i = 0; i < s->count; ++i) {
        VC* vc = s->vcs + i; PC* pc = s->pcs + i;
        float radiusA = pc->radiusA, radiusB = pc->radiusB;
        Manifold* manifold = &s->contacts[vc->contactIndex]->manifold;
        int indexA = vc->indexA, indexB = vc->indexB;
        float mA = vc->invMassA, mB = vc->invMassB, iA = vc->invIA, iB = vc->invIB;
        V2 localCenterA = pc->localCenterA, localCenterB = pc->localCenterB;
        V2 cA = s->positions[indexA].c; float aA = s->positions[indexA].a;
        V2 vA = s->velocities[indexA].v; float wA = s->velocities[indexA].w;
        V2 cB = s->positions[indexB].c; float aB = s->positions[indexB].a;
        V2 vB = s->velocities[indexB].v; float wB = s->velocities[indexB].w;
        Xf xfA, xfB;
        xfA.q = rot(aA); xfB.q = rot(aB);
        xfA.p = vsub(cA, mul_rv(xfA.q, localCenterA));
        xfB.p = vsub(cB, mul_rv(xfB.q, localCenterB));
        V2 wmNormal = v2(0.0f, 0.0f); V2 wmPoints[2];
        world_manifold(manifold, xfA, radiusA, xfB, radiusB, &wmNormal, wmPoints);
        vc->normal = wmNormal;
        int pointCount = vc->pointCount;
        for (int j = 0; j < pointCount; ++j) {
            VCPoint* vcp = vc->points + j;
            vcp->rA = vsub(wmPoints[j], cA);
            vcp->rB = vsub(wmPoints[j], cB);
            float rnA = vcross(vcp->rA, vc->normal);
            float rnB = vcross(vcp->rB, vc->normal);
            float kNormal = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
            vcp->normalMass = kNormal > 0.0f ? 1.0f / kNormal : 0.0f;
            V2 tangent = vcross_vs(vc->normal, 1.0f);
            float rtA = vcross(vcp->rA, tangent);
            float rtB = vcross(vcp->rB, tangent);
            float kTangent = mA + mB + iA * rtA * rtA + iB * rtB * rtB;
            vcp->tangentMass = kTangent > 0.0f ? 1.0f / kTangent : 0.0f;
            vcp->velocityBias = 0.0f;
            V2 dvr = vsub(vsub(vadd(vB, vcross_sv(wB, vcp->rB)), vA), vcross_sv(wA, vcp->rA));
            float vRel = vdot(vc->normal, dvr);
            if (vRel < -VELOCITY_THRESHOLD) vcp->velocityBias = -vc->restitution * vRel;
        }
        if (vc->pointCount == 2) {
            VCPoint* vcp1 = vc->points + 0; VCPoint* vcp2 = vc->points + 1;
            float rn1A = vcross(vcp1->rA, vc->normal), rn1B = vcross(vcp1->rB, vc->normal);
            float rn2A = vcross(vcp2->rA, vc->normal), rn2B = vcross(vcp2->rB, vc->normal);
            float k11 = mA + mB + iA * rn1A * rn1A + iB * rn1B * rn1B;
            float k22 = mA + mB + iA * rn2A * rn2A + iB * rn2B * rn2B;
            float k12 = mA + mB + iA * rn1A * rn2A + iB * rn1B * rn2B;
            const float k_maxConditionNumber = 1000.0f;
            if (k11 * k11 < k_maxConditionNumber * (k11 * k22 - k12 * k12)) {
                vc->K[0] = k11; vc->K[1] = k12; vc->K[2] = k12; vc->K[3] = k22;   /* ex=(k11,k12) ey=(k12,k22) */
                float a = vc->K[0], b = vc->K[2], c = vc->K[1], d = vc->K[3];
                float det = a * d - b * c;
                if (det != 0.0f) det = 1.0f / det;
                vc->nm[0] = det * d; vc->nm[2] = -det * b;   /* ex.x, ey.x */
                vc->nm[1] = -det * c; vc->nm[3] = det * a;   /* ex.y, ey.y */
            } else {
                vc->pointCount = 1;
            }
        }
    }
}

static void solver_warm_start(Solver* s) {
    for (int i = 0; i < s->count; ++i) {
        VC* vc = s->vcs + i;
        int indexA = vc->indexA, indexB = vc->indexB;
        float mA = vc->invMassA, iA = vc->invIA, mB = vc->invMassB, iB = vc->invIB;
        int pointCount = vc->pointCount;
        V2 vA = s->velocities[indexA].v; float wA = s->velocities[indexA].w;
        V2 vB = s->velocities[indexB].v; float wB = s->velocities[indexB].w;
        V2 normal = vc->normal; V2 tangent = vcross_vs(normal, 1.0f);
        for (int j = 0; j < pointCount; ++j) {
            VCPoint* vcp = vc->points + j;
            V2 P = vadd(vmul(vcp->normalImpulse, normal), vmul(vcp->tangentImpulse, tangent));
            wA -= iA * vcross(vcp->rA, P);
            vA = vsub(vA, vmul(mA, P));
            wB += iB * vcross(vcp->rB, P);
            vB = vadd(vB, vmul(mB, P));
        }
        s->velocities[indexA].v = vA; s->velocities[indexA].w = wA;
        s->velocities[indexB].v = vB; s->velocities[indexB].w = wB;
    }
}

static inline V2 mat_mul(const float* M, V2 v) {   /* M = {ex.x, ex.y, ey.x, ey.y} */
    return v2(M[0] * v.x + M[2] * v.y, M[1] * v.x + M[3] * v.y);
}

/* diagnostic (b2o_lcp_cases): how often each case of the 2-point block solver applies (cases 1-4,
 * then "no solution"), counted over every 2-point velocity update since the last reset; plus the
 * 1-point updates and the updates whose normal impulses are subnormal (tools: chain analysis) */
#ifndef OR_NO_WORK
static long g_lcp[8];
#define LCP_CASE(k) do { _Pragma("omp atomic") g_lcp[k]++; } while (0)
void b2o_lcp_cases(long* out8, int reset) {
    for (int k = 0; k < 8; ++k) { if (out8) out8[k] = g_lcp[k]; if (reset) g_lcp[k] = 0; }
}
#else
#define LCP_CASE(k) do {} while (0)
#endif
static void solver_solve_velocity(Solver* s) {
    for (int i = 0; i < s->count; ++i) {
        VC* vc = s->vcs + i;
        int indexA = vc->indexA, indexB = vc->indexB;
        float mA = vc->invMassA, iA = vc->invIA, mB = vc->invMassB, iB = vc->invIB;
        int pointCount = vc->pointCount;
        V2 vA = s->velocities[indexA].v; float wA = s->velocities[indexA].w;
        V2 vB = s->velocities[indexB].v; float wB = s->velocities[indexB].w;
        V2 normal = vc->normal; V2 tangent = vcross_vs(normal, 1.0f);
        float friction = vc->friction;
        for (int j = 0; j < pointCount; ++j) {
            VCPoint* vcp = vc->points + j;
            V2 dv = vsub(vsub(vadd(vB, vcross_sv(wB, vcp->rB)), vA), vcross_sv(wA, vcp->rA));
            float vt = vdot(dv, tangent) - vc->tangentSpeed;
            float lambda = vcp->tangentMass * (-vt);
            float maxFriction = friction * vcp->normalImpulse;
            float newImpulse = fclamp(vcp->tangentImpulse + lambda, -maxFriction, maxFriction);
            lambda = newImpulse - vcp->tangentImpulse;
            vcp->tangentImpulse = newImpulse;
            V2 P = vmul(lambda, tangent);
            vA = vsub(vA, vmul(mA, P));
            wA -= iA * vcross(vcp->rA, P);
            vB = vadd(vB, vmul(mB, P));
            wB += iB * vcross(vcp->rB, P);
        }
        if (vc->pointCount == 1) {
            VCPoint* vcp = vc->points + 0;
            V2 dv = vsub(vsub(vadd(vB, vcross_sv(wB, vcp->rB)), vA), vcross_sv(wA, vcp->rA));
            float vn = vdot(dv, normal);
            float lambda = -vcp->normalMass * (vn - vcp->velocityBias);
            float newImpulse = fmax_(vcp->normalImpulse + lambda, 0.0f);
            lambda = newImpulse - vcp->normalImpulse;
            vcp->normalImpulse = newImpulse;
            V2 P = vmul(lambda, normal);
            vA = vsub(vA, vmul(mA, P));
            wA -= iA * vcross(vcp->rA, P);
            vB = vadd(vB, vmul(mB, P));
            wB += iB * vcross(vcp->rB, P);
        } else {
            VCPoint* cp1 = vc->points + 0; VCPoint* cp2 = vc->points + 1;
            V2 a = v2(cp1->normalImpulse, cp2->normalImpulse);
            V2 dv1 = vsub(vsub(vadd(vB, vcross_sv(wB, cp1->rB)), vA), vcross_sv(wA, cp1->rA));
            V2 dv2 = vsub(vsub(vadd(vB, vcross_sv(wB, cp2->rB)), vA), vcross_sv(wA, cp2->rA));
            float vn1 = vdot(dv1, normal), vn2 = vdot(dv2, normal);
            V2 b; b.x = vn1 - cp1->velocityBias; b.y = vn2 - cp2->velocityBias;
            b = vsub(b, mat_mul(vc->K, a));
            for (;;) {
                V2 x = vneg(mat_mul(vc->nm, b));
                if (x.x >= 0.0f && x.y >= 0.0f) { LCP_CASE(0); goto apply; }
                x.x = -cp1->normalMass * b.x; x.y = 0.0f;
                vn1 = 0.0f; vn2 = vc->K[1] * x.x + b.y;
                if (x.x >= 0.0f && vn2 >= 0.0f) { LCP_CASE(1); goto apply; }
                x.x = 0.0f; x.y = -cp2->normalMass * b.y;
                vn1 = vc->K[2] * x.y + b.x; vn2 = 0.0f;
                if (x.y >= 0.0f && vn1 >= 0.0f) { LCP_CASE(2); goto apply; }
                x.x = 0.0f; x.y = 0.0f; vn1 = b.x; vn2 = b.y;
                if (vn1 >= 0.0f && vn2 >= 0.0f) { LCP_CASE(3); goto apply; }
                LCP_CASE(4);
                break;
            apply: {
                    V2 d = vsub(x, a);
                    V2 P1 = vmul(d.x, normal), P2 = vmul(d.y, normal);
                    vA = vsub(vA, vmul(mA, vadd(P1, P2)));
                    wA -= iA * (vcross(cp1->rA, P1) + vcross(cp2->rA, P2));
                    vB = vadd(vB, vmul(mB, vadd(P1, P2)));
                    wB += iB * (vcross(cp1->rB, P1) + vcross(cp2->rB, P2));
                    cp1->normalImpulse = x.x; cp2->normalImpulse = x.y;
                    break;
                }
            }
        }
        s->velocities[indexA].v = vA; s->velocities[indexA].w = wA;
        s->velocities[indexB].v = vB; s->velocities[indexB].w = wB;
    }
}

static void solver_store_impulses(Solver* s) {
    for (int i = 0; i < s->count; ++i) {
        VC* vc = s->vcs + i;
        Manifold* m = &s->contacts[vc->contactIndex]->manifold;
        for (int j = 0; j < vc->pointCount; ++j) {
            m->points[j].normalImpulse = vc->points[j].normalImpulse;
            m->points[j].tangentImpulse = vc->points[j].tangentImpulse;
        }
    }
}

static void psm_init(const PC* pc, Xf xfA, Xf xfB, int index, V2* normal, V2* point, float* separation) {
    if (pc->type == MT_FACEA) {
        *normal = mul_rv(xfA.q, pc->localNormal);
        V2 planePoint = mul_xv(xfA, pc->localPoint);
        V2 clipPoint = mul_xv(xfB, pc->localPoints[index]);
        *separation = vdot(vsub(clipPoint, planePoint), *normal) - pc->radiusA - pc->radiusB;
        *point = clipPoint;
    } else {
        *normal = mul_rv(xfB.q, pc->localNormal);
        V2 planePoint = mul_xv(xfB, pc->localPoint);
        V2 clipPoint = mul_xv(xfA, pc->localPoints[index]);
        *separation = vdot(vsub(clipPoint, planePoint), *normal) - pc->radiusA - pc->radiusB;
        *point = clipPoint;
        *normal = vneg(*normal);
    }
}

static int solver_solve_position(Solver* s, int toi, int toiIndexA, int toiIndexB) {
    float minSeparation = 0.0f;
    for (int i = 0; i < s->count; ++i) {
        PC* pc = s->pcs + i;
        int indexA = pc->indexA, indexB = pc->indexB;
        V2 localCenterA = pc->localCenterA, localCenterB = pc->localCenterB;
        int pointCount = pc->pointCount;
        float mA, iA, mB, iB;
        if (!toi) {
            mA = pc->invMassA; iA = pc->invIA; mB = pc->invMassB; iB = pc->invIB;
        } else {
            mA = 0.0f; iA = 0.0f;
            if (indexA == toiIndexA || indexA == toiIndexB) { mA = pc->invMassA; iA = pc->invIA; }
            mB = 0.0f; iB = 0.0f;
            if (indexB == toiIndexA || indexB == toiIndexB) { mB = pc->invMassB; iB = pc->invIB; }
        }
        V2 cA = s->positions[indexA].c; float aA = s->positions[indexA].a;
        V2 cB = s->positions[indexB].c; float aB = s->positions[indexB].a;
        for (int j = 0; j < pointCount; ++j) {
            Xf xfA, xfB;
            xfA.q = rot(aA); xfB.q = rot(aB);
            xfA.p = vsub(cA, mul_rv(xfA.q, localCenterA));
            xfB.p = vsub(cB, mul_rv(xfB.q, localCenterB));
            V2 normal, point; float separation;
            psm_init(pc, xfA, xfB, j, &normal, &point, &separation);
            V2 rA = vsub(point, cA), rB = vsub(point, cB);
            minSeparation = fmin_(minSeparation, separation);
            float C = fclamp((toi ? TOI_BAUMGARTE : BAUMGARTE) * (separation + LINEAR_SLOP), -MAX_LINEAR_CORRECTION, 0.0f);
            float rnA = vcross(rA, normal), rnB = vcross(rB, normal);
            float K = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
            float impulse = K > 0.0f ? -C / K : 0.0f;
            V2 P = vmul(impulse, normal);
            cA = vsub(cA, vmul(mA, P));
            aA -= iA * vcross(rA, P);
            cB = vadd(cB, vmul(mB, P));
            aB += iB * vcross(rB, P);
        }
        s->positions[indexA].c = cA; s->positions[indexA].a = aA;
        s->positions[indexB].c = cB; s->positions[indexB].a = aB;
    }
    return toi ? (minSeparation >= -1.5f * LINEAR_SLOP) : (minSeparation >= -3.0f * LINEAR_SLOP);
}

/* ---------------------------------------------------------------- island [B2 b2Island.cpp] */
typedef struct {
    Body** bodies; Contact** contacts; Position* positions; Velocity* velocities;
    int bodyCount, contactCount, bodyCapacity, contactCapacity;
} Island;

static void island_init(Island* is, int bodyCap, int contactCap) {
    is->bodyCapacity = bodyCap; is->contactCapacity = contactCap;
    is->bodies = (Body**)calloc((size_t)(bodyCap + 1), sizeof(Body*));
    is->contacts = (Contact**)calloc((size_t)(contactCap + 1), sizeof(Contact*));
    is->positions = (Position*)calloc((size_t)(bodyCap + 1), sizeof(Position));
    is->velocities = (Velocity*)calloc((size_t)(bodyCap + 1), sizeof(Velocity));
    is->bodyCount = 0; is->contactCount = 0;
}
static void island_free(Island* is) { free(is->bodies); free(is->contacts); free(is->positions); free(is->velocities); }
static void island_add_body(Island* is, Body* b) { b->islandIndex = is->bodyCount; is->bodies[is->bodyCount++] = b; }
static void island_add_contact(Island* is, Contact* c) { is->contacts[is->contactCount++] = c; }

static void integrate_positions(Island* is, float h, int syncBodies) {
    for (int i = 0; i < is->bodyCount; ++i) {
        V2 c = is->positions[i].c; float a = is->positions[i].a;
        V2 v = is->velocities[i].v; float w = is->velocities[i].w;
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
        is->positions[i].c = c; is->positions[i].a = a;
        is->velocities[i].v = v; is->velocities[i].w = w;
        if (syncBodies) {
            Body* body = is->bodies[i];
            body->sweep.c = c; body->sweep.a = a; body->v = v; body->w = w;
            body_synchronize_transform(body);
        }
    }
}

/* ---- work model (OrWork, test infrastructure): device sweep counts and dependency levels ---- */
/* dependency levels of the island's Gauss-Seidel order: contact i waits for the last earlier
 * contact that shares one of its dynamic bodies (`dyn[k]`: island body k moves under this solve);
 * returns the level count, and the sum over levels of each level's largest point count */
static int work_levels(const Solver* s, const int* dyn, int* level_points) {
    int last[256], lvmax_pts[256];
    int nb = 0;
    for (int i = 0; i < s->count; ++i) {
        const int a = s->vcs[i].indexA, b = s->vcs[i].indexB;
        if (a + 1 > nb) nb = a + 1;
        if (b + 1 > nb) nb = b + 1;
    }
    for (int k = 0; k < nb && k < 256; ++k) last[k] = 0;
    int L = 0;
    for (int i = 0; i < s->count && i < 256; ++i) {
        const int a = s->vcs[i].indexA, b = s->vcs[i].indexB;
        int lv = 1;
        if (dyn[a] && last[a] + 1 > lv) lv = last[a] + 1;
        if (dyn[b] && last[b] + 1 > lv) lv = last[b] + 1;
        if (dyn[a]) last[a] = lv;
        if (dyn[b]) last[b] = lv;
        if (lv > L) { for (int k = L; k < lv; ++k) lvmax_pts[k] = 0; L = lv; }
        if (s->pcs[i].pointCount > lvmax_pts[lv - 1]) lvmax_pts[lv - 1] = s->pcs[i].pointCount;
    }
    int lp = 0;
    for (int k = 0; k < L; ++k) lp += lvmax_pts[k];
    if (level_points) *level_points = lp;
    return L;
}
/* critical path of `reps` repetitions of the island's Gauss-Seidel order, each contact lasting
 * its point count (by_points) or 1: a contact starts when the previous contacts that share one of
 * its dynamic bodies have finished (the sweeps unrolled, so sweep k+1 may overlap sweep k) */
static long work_pipe(const Solver* s, const int* dyn, int reps, int by_points) {
    long fin[256];
    int nb = 0;
    for (int i = 0; i < s->count; ++i) {
        if (s->vcs[i].indexA + 1 > nb) nb = s->vcs[i].indexA + 1;
        if (s->vcs[i].indexB + 1 > nb) nb = s->vcs[i].indexB + 1;
    }
    for (int k = 0; k < nb && k < 256; ++k) fin[k] = 0;
    long end = 0;
    for (int r = 0; r < reps; ++r)
        for (int i = 0; i < s->count; ++i) {
            const int a = s->vcs[i].indexA, b = s->vcs[i].indexB;
            long t = 0;
            if (dyn[a] && fin[a] > t) t = fin[a];
            if (dyn[b] && fin[b] > t) t = fin[b];
            t += by_points ? s->pcs[i].pointCount : 1;
            if (dyn[a]) fin[a] = t;
            if (dyn[b]) fin[b] = t;
            if (t > end) end = t;
        }
    return end;
}
/* the velocity sweeps with the device's exact early-exit count: the sweep loop always runs all
 * `iters` (results are the reference's), the return value is the number the device runs */
/* diagnostic (b2o_period_diag): for islands whose sweeps never reach period 1 or 2, the earliest
 * sweep at which the state repeats with ANY period up to 64, histogrammed; [0] islands examined,
 * [1] of them with no repeat within `iters`, [2 + k] first repeat at sweep k (k < 190), and the
 * period histogram at [200 + p] */
static int g_period_diag = 0;
static long g_period_hist[300];
void b2o_period_diag(int on, long* out300) {
    if (out300) for (int i = 0; i < 300; ++i) out300[i] = g_period_hist[i];
    if (on >= 0) { g_period_diag = on; for (int i = 0; i < 300; ++i) g_period_hist[i] = 0; }
}
static int g_model_period = 0;   /* > 0: the work model counts sweeps as if periods up to this were detected */
void b2o_model_period(int p) { g_model_period = p; }
static int period_scan(const float* hist, int ns, int iters) {
    int first = -1, per = 0;
    const int pmax = g_model_period > 0 ? g_model_period : 64;
    for (int k = 1; k <= iters && first < 0; ++k)
        for (int p = 1; p <= pmax && p <= k; ++p)
            if (memcmp(hist + (size_t)k * ns, hist + (size_t)(k - p) * ns, sizeof(float) * (size_t)ns) == 0) {
                first = k; per = p; break;
            }
#pragma omp critical
    {
        g_period_hist[0]++;
        if (first < 0) g_period_hist[1]++;
        else { g_period_hist[2 + (first < 190 ? first : 189)]++; g_period_hist[200 + per]++; }
    }
    return first;
}

/* The device's early-exit compare schedule (mrp_world.h exit_mask, MRP_EXIT_DENSE = 32 /
 * MRP_EXIT_SPARSE = 16): after sweep `done` the state is compared with the snapshot of two sweeps
 * earlier when (iters - done) & mask == 0 and snapshotted when it is 2.  One definition for the work
 * model (the device sweep counts of tools/roofline_model.py) and the early-exit CPU port. */
#define OR_EXIT_DENSE 32
#define OR_EXIT_SPARSE 16
static inline int exit_mask(int done) { return done > OR_EXIT_DENSE ? OR_EXIT_SPARSE - 1 : 3; }

static int work_velocity_sweeps(Solver* s, int iters, int nbodies) {
    const int nc = s->count, ns = 4 * nc + 3 * nbodies;
    float* snap = (float*)malloc(sizeof(float) * (size_t)(ns > 0 ? ns : 1));
    float* cur = (float*)malloc(sizeof(float) * (size_t)(ns > 0 ? ns : 1));
#define WORK_STATE(dst) do {                                                                       \
        int k_ = 0;                                                                                \
        for (int i_ = 0; i_ < nc; ++i_)                                                            \
            for (int j_ = 0; j_ < 2; ++j_) {                                                       \
                (dst)[k_++] = s->vcs[i_].points[j_].normalImpulse;                                 \
                (dst)[k_++] = s->vcs[i_].points[j_].tangentImpulse;                                \
            }                                                                                      \
        for (int b_ = 0; b_ < nbodies; ++b_) {                                                     \
            (dst)[k_++] = s->velocities[b_].v.x; (dst)[k_++] = s->velocities[b_].v.y;              \
            (dst)[k_++] = s->velocities[b_].w;                                                     \
        }                                                                                          \
    } while (0)
    int have = (iters & 3) == 2, run = -1;
    if (have) WORK_STATE(snap);
    float* hist = (g_period_diag || g_model_period > 0) ? (float*)malloc(sizeof(float) * (size_t)(ns > 0 ? ns : 1) * (size_t)(iters + 1)) : NULL;
    if (hist) WORK_STATE(hist);
    for (int it = 0; it < iters; ++it) {
        solver_solve_velocity(s);
        if (hist) WORK_STATE(hist + (size_t)(it + 1) * ns);
        if (run >= 0) continue;
        const int left = iters - (it + 1), m = exit_mask(it + 1);
        if ((left & m) == 0 && have) {
            WORK_STATE(cur);
            if (memcmp(cur, snap, sizeof(float) * (size_t)ns) == 0) run = it + 1;
        }
        if ((left & m) == 2) { WORK_STATE(snap); have = 1; }
    }
#undef WORK_STATE
    if (hist) {
        if (run < 0 && nc > 0) {
            const int first = period_scan(hist, ns, iters);
            if (g_model_period > 0 && first > 0) run = first;
        }
        free(hist);
    }
    free(snap);
    free(cur);
    return run >= 0 ? run : iters;
}

/* diagnostic (b2o_model_2wave): the island's `sweeps` velocity sweeps (device
 * count, `iters` configured) priced on one wave, and split over two waves of one workgroup.  Each
 * wave runs its contacts in the island's Gauss-Seidel order; a contact starts when its wave is free
 * and every dynamic body it touches holds the value of the body's previous update in sequential order
 * (+x cycles when that update ran on the other wave: an LDS handoff), so the split is bit-exact by
 * construction.  At each early-exit compare point the waves meet (+b).  The partition (contact 0 on
 * wave 0) is the best of all 2^(nc-1) for nc <= 12 over the first min(sweeps, 8) sweeps. */
static double g2w_cost[16], g2w_x = -1.0, g2w_b = 0.0, g2w_read = 0.0, g2w_pub = 0.0;
void b2o_model_2wave(const double* cost16, double x, double b) {
    if (!cost16) { g2w_x = -1.0; return; }
    /* OR_2W_READ / OR_2W_PUB: cycles a cross-wave dependency adds to the consumer's update (its LDS
     * read of the body) and to the producer's (the LDS write + flag), waiting or not */
    g2w_read = getenv("OR_2W_READ") ? atof(getenv("OR_2W_READ")) : 0.0;
    g2w_pub = getenv("OR_2W_PUB") ? atof(getenv("OR_2W_PUB")) : 0.0;
    for (int i = 0; i < 16; ++i) g2w_cost[i] = cost16[i];
    g2w_x = x; g2w_b = b;
}
static double twowave_run(const Solver* s, const int* dyn, int nb, unsigned mask, int sweeps, int iters, int barriers) {
    double fin[256], tw[2] = {0.0, 0.0};
    int own[256], n[2] = {0, 0};
    for (int i = 0; i < s->count; ++i) ++n[(mask >> i) & 1u];
    for (int k = 0; k < nb; ++k) { fin[k] = 0.0; own[k] = -1; }
    int have = (iters & 3) == 2;
    for (int r = 0; r < sweeps; ++r) {
        for (int i = 0; i < s->count; ++i) {
            const int w = (mask >> i) & 1u, ab[2] = {s->vcs[i].indexA, s->vcs[i].indexB};
            double t = tw[w], rd = 0.0, pub = 0.0;
            for (int j = 0; j < 2; ++j)
                if (dyn[ab[j]] && own[ab[j]] >= 0) {
                    const double ready = fin[ab[j]] + (own[ab[j]] != w ? g2w_x : 0.0);
                    if (own[ab[j]] != w) rd = g2w_read;   /* the LDS read of a body the other wave wrote */
                    if (ready > t) t = ready;
                }
            for (int j = 0; j < 2 && mask; ++j)   /* publishing a body the other wave updates next */
                if (dyn[ab[j]]) {
                    int nx = -1;
                    for (int q = 1; q <= s->count && nx < 0; ++q) {
                        const int k2 = (i + q) % s->count;
                        if (s->vcs[k2].indexA == ab[j] || s->vcs[k2].indexB == ab[j]) nx = k2;
                    }
                    if (nx >= 0 && (int)((mask >> nx) & 1u) != w) pub = g2w_pub;
                }
            const int nw = n[w] < 8 ? n[w] : 8, p = s->vcs[i].pointCount < 2 ? 0 : 1;
            t += rd + pub + g2w_cost[p * 8 + nw - 1];
            tw[w] = t;
            for (int j = 0; j < 2; ++j)
                if (dyn[ab[j]]) { fin[ab[j]] = t; own[ab[j]] = w; }
        }
        if (!barriers) continue;
        const int done = r + 1, left = iters - done, m = exit_mask(done);
        if ((left & m) == 0 && have) {
            const double t = (tw[0] > tw[1] ? tw[0] : tw[1]) + g2w_b;
            tw[0] = tw[1] = t;
        }
        if ((left & m) == 2) have = 1;
    }
    return tw[0] > tw[1] ? tw[0] : tw[1];
}
/* Paired contact updates on one wave (b2o_model_dual): the island's Gauss-Seidel stream of
 * `D` sweeps (item q = sweep q / nc, contact q % nc) cut into slots of one or two updates run by one
 * instruction stream in two lanes.  Greedy, in stream order: a slot takes the first unscheduled item
 * u and the first unscheduled item v after it (at most `window` items on) with u's point count that
 * shares no dynamic body with u nor with any unscheduled item between them -- so every body and
 * every contact sees its updates in the sequential order and the result is bit-exact.  out[t] =
 * u | v << 4 (v == u: a single); returns the slot count (or -1 when `cap` is too small). */
static int g_dual_mixed = 0;   /* model only: pairs of any point counts */
int b2o_dual_schedule(int nc, const int* ia, const int* ib, const int* dyn, const int* pcount, int D, int window,
                      unsigned char* out, int cap) {
    const int n = nc * D;
    unsigned char done[2048];
    if (n > 2048 || nc > 15) return -1;
    for (int q = 0; q < n; ++q) done[q] = 0;
    int t = 0, u = 0;
#define CONFL(p, q) ((dyn[ia[(p) % nc]] && (ia[(p) % nc] == ia[(q) % nc] || ia[(p) % nc] == ib[(q) % nc])) || \
                     (dyn[ib[(p) % nc]] && (ib[(p) % nc] == ia[(q) % nc] || ib[(p) % nc] == ib[(q) % nc])))
    while (u < n) {
        done[u] = 1;
        int v = u;
        for (int q = u + 1; q < n && q <= u + window; ++q) {
            if (done[q] || (!g_dual_mixed && pcount[q % nc] != pcount[u % nc]) || CONFL(u, q)) continue;
            int ok = 1;
            for (int r = u + 1; r < q && ok; ++r)
                if (!done[r] && CONFL(r, q)) ok = 0;
            if (ok) { v = q; break; }
        }
        done[v] = 1;
        if (t >= cap) return -1;
        out[t++] = (unsigned char)((u % nc) | ((v % nc) << 4));
        while (u < n && done[u]) ++u;
    }
#undef CONFL
    return t;
}
static double g_dual_factor = 0.0;
static int g_dual_window = 0, g_dual_nodrain = 0;
/* window < 0: |window|, and the stream never drains (the bound without early-exit meeting points) */
void b2o_model_dual(double factor, int window) {
    g_dual_factor = factor; g_dual_window = window < 0 ? -window : window; g_dual_nodrain = window < 0;
    g_dual_mixed = getenv("OR_DUAL_MIXED") != NULL;
}
/* the sweeps as the paired path would run them: segments between the early-exit events (snapshot
 * and compare sweeps, where the stream drains), each slot priced as one update x factor */
static double dual_run(const Solver* s, const int* dyn, int sweeps, int iters) {
    const int nc = s->count;
    int ia[16], ib[16], pc[16];
    for (int i = 0; i < nc; ++i) { ia[i] = s->vcs[i].indexA; ib[i] = s->vcs[i].indexB; pc[i] = s->vcs[i].pointCount; }
    unsigned char sl[2048];
    double t = 0.0;
    int k = 0;
    while (k < sweeps) {
        int e = g_dual_nodrain ? sweeps : k + 1;   /* next event sweep (or the end) */
        while (e < sweeps) {
            const int left = iters - e, m = exit_mask(e);
            if ((left & m) == 0 || (left & m) == 2) break;
            ++e;
        }
        const int D = e - k;
        const int ns = b2o_dual_schedule(nc, ia, ib, dyn, pc, D, g_dual_window, sl, 2048);
        if (ns < 0) return -1.0;
        for (int q = 0; q < ns; ++q) {
            const int u = sl[q] & 15, p = pc[u] < 2 ? 0 : 1;
            t += g2w_cost[p * 8 + (nc < 8 ? nc : 8) - 1] * g_dual_factor;
        }
        k = e;
    }
    return t;
}
static void work_model_2wave(const Solver* s, const int* dyn, int sweeps, int iters, OrWork* k) {
    if (g2w_x < 0.0 || s->count < 1) return;
    if (g_dual_factor > 0.0) {   /* b2o_model_dual: vel_2wave holds the paired one-wave path */
        const double one = twowave_run(s, dyn, 256, 0u, sweeps, iters, 0);
        double d = s->count >= 3 && s->count <= 15 ? dual_run(s, dyn, sweeps, iters) : one;
        if (d < 0.0) d = one;
        k->vel_1wave += (long)(one + 0.5);
        k->vel_2wave += (long)(d + 0.5);
        return;
    }
    int nb = 0;
    for (int i = 0; i < s->count; ++i) {
        if (s->vcs[i].indexA + 1 > nb) nb = s->vcs[i].indexA + 1;
        if (s->vcs[i].indexB + 1 > nb) nb = s->vcs[i].indexB + 1;
    }
    if (nb > 256) return;
    const double one = twowave_run(s, dyn, nb, 0u, sweeps, iters, 0);
    double two = one;
    if (s->count >= 2 && s->count <= 12) {
        unsigned best = 0u;
        double bt = 0.0;
        const int probe = sweeps < 8 ? sweeps : 8;
        for (unsigned m = 0; m < (1u << (s->count - 1)); ++m) {
            const unsigned mask = m << 1;   /* contact 0 stays on wave 0 */
            const double t = twowave_run(s, dyn, nb, mask, probe, iters, 0);
            if (m == 0 || t < bt) { bt = t; best = mask; }
        }
        two = twowave_run(s, dyn, nb, best, sweeps, iters, 1);
        if (best == 0u || two > one) two = one;   /* a split that does not pay stays on one wave */
    }
    k->vel_1wave += (long)(one + 0.5);
    k->vel_2wave += (long)(two + 0.5);
}

/* diagnostic (b2o_topo_diag(1); b2o_topo_diag(2) also records 1- and 2-contact islands): island
 * topologies of 3- and 4-contact islands, weighted by sweeps run:
 * per contact (A slot, B slot, point count) with body slots numbered by first appearance and static
 * bodies as slot 7; 64 distinct signatures kept */
static int g_topo_diag = 0;
static long g_topo_sig[64], g_topo_w[64];
static void topo_record(const Solver* s, const Island* is, int sweeps) {
    int slot[256], ns = 0;
    for (int k = 0; k < 256; ++k) slot[k] = -1;
    long sig = s->count;
    for (int i = 0; i < s->count; ++i) {
        const int ab[2] = {s->vcs[i].indexA, s->vcs[i].indexB};
        int sl[2];
        for (int j = 0; j < 2; ++j) {
            const Body* b = is->bodies[ab[j]];
            if (b->invMass == 0.0f && b->invI == 0.0f) { sl[j] = 7; continue; }
            if (slot[ab[j]] < 0) slot[ab[j]] = ns++;
            sl[j] = slot[ab[j]];
        }
        sig = sig * 1000 + sl[0] * 100 + sl[1] * 10 + s->vcs[i].pointCount;
    }
#pragma omp critical
    {
        int k = 0;
        while (k < 64 && g_topo_w[k] && g_topo_sig[k] != sig) ++k;
        if (k < 64) { g_topo_sig[k] = sig; g_topo_w[k] += sweeps * (long)s->count; }
    }
}
/* b2o_topo_diag(3): print (stderr, first 60) the contact list of islands with >= 5 contacts that run
 * >= 100 sweeps: per contact "A-B/points", body slots by first appearance, static bodies as S */
static int g_topo_printed = 0;
static void topo_print(const Solver* s, const Island* is, int sweeps) {
    char buf[512];
    int slot[256], ns = 0, n = 0;
    for (int k = 0; k < 256; ++k) slot[k] = -1;
    n += snprintf(buf + n, sizeof(buf) - n, "nc %d sweeps %3d:", s->count, sweeps);
    for (int i = 0; i < s->count && n < 480; ++i) {
        const int ab[2] = {s->vcs[i].indexA, s->vcs[i].indexB};
        char c[2];
        for (int j = 0; j < 2; ++j) {
            const Body* b = is->bodies[ab[j]];
            if (b->invMass == 0.0f && b->invI == 0.0f) { c[j] = 'S'; continue; }
            if (slot[ab[j]] < 0) slot[ab[j]] = ns++;
            c[j] = (char)('0' + slot[ab[j]]);
        }
        n += snprintf(buf + n, sizeof(buf) - n, " %c-%c/%d", c[0], c[1], s->vcs[i].pointCount);
    }
#pragma omp critical
    {
        if (g_topo_printed < 100000) { fprintf(stderr, "%s\n", buf); ++g_topo_printed; }
    }
}
void b2o_topo_diag(int on, long* sig64, long* w64) {
    g_topo_printed = 0;
    for (int k = 0; k < 64; ++k) { if (sig64) sig64[k] = g_topo_sig[k]; if (w64) w64[k] = g_topo_w[k]; }
    if (on >= 0) { g_topo_diag = on; for (int k = 0; k < 64; ++k) { g_topo_sig[k] = 0; g_topo_w[k] = 0; } }
}

#ifdef OR_NO_WORK
/* CPU-baseline builds (Makefile targets `fast` and `early`, bench.py cpu_baseline): the velocity
 * sweeps without the work model.  OR_EARLY_EXIT stops at the device's exact early exit
 * (mrp_world.h solver_velocity_*): a snapshot two sweeps before every sweep k with 180 - k = 0
 * (mod 4 up to sweep 32, mod 16 after), and once the state after k equals it the state has period
 * 1 or 2, so the state after
 * all `iters` sweeps is the state after k -- the same bits, fewer sweeps.  Without OR_EARLY_EXIT
 * all `iters` sweeps run, as b2ContactSolver::SolveVelocityConstraints is called by b2Island::Solve. */
static void velocity_sweeps(Solver* s, int iters, int nbodies) {
#ifdef OR_EARLY_EXIT
    const int nc = s->count, ns = 4 * nc + 3 * nbodies;
    float snap_st[512], cur_st[512];
    float* snap = ns <= 512 ? snap_st : (float*)malloc(sizeof(float) * (size_t)ns);
    float* cur = ns <= 512 ? cur_st : (float*)malloc(sizeof(float) * (size_t)ns);
#define SWEEP_STATE(dst) do {                                                                      \
        int k_ = 0;                                                                                \
        for (int i_ = 0; i_ < nc; ++i_)                                                            \
            for (int j_ = 0; j_ < 2; ++j_) {                                                       \
                (dst)[k_++] = s->vcs[i_].points[j_].normalImpulse;                                 \
                (dst)[k_++] = s->vcs[i_].points[j_].tangentImpulse;                                \
            }                                                                                      \
        for (int b_ = 0; b_ < nbodies; ++b_) {                                                     \
            (dst)[k_++] = s->velocities[b_].v.x; (dst)[k_++] = s->velocities[b_].v.y;              \
            (dst)[k_++] = s->velocities[b_].w;                                                     \
        }                                                                                          \
    } while (0)
    int have = (iters & 3) == 2;
    if (have) SWEEP_STATE(snap);
    for (int it = 0; it < iters; ++it) {
        solver_solve_velocity(s);
        /* the device's schedule (mrp_world.h exit_mask): every 4 sweeps up to sweep 32, then every 16 */
        const int left = iters - (it + 1), m = exit_mask(it + 1);
        if ((left & m) == 0 && have) {
            SWEEP_STATE(cur);
            if (memcmp(cur, snap, sizeof(float) * (size_t)ns) == 0) break;
        }
        if ((left & m) == 2) { SWEEP_STATE(snap); have = 1; }
    }
#undef SWEEP_STATE
    if (snap != snap_st) free(snap);
    if (cur != cur_st) free(cur);
#else
    (void)nbodies;
    for (int it = 0; it < iters; ++it) solver_solve_velocity(s);
#endif
}
#endif

static void island_solve(Island* is, World* w, TimeStep step) {
    float h = step.dt;
    for (int i = 0; i < is->bodyCount; ++i) {
        Body* b = is->bodies[i];
        V2 c = b->sweep.c; float a = b->sweep.a;
        V2 v = b->v; float wv = b->w;
        b->sweep.c0 = b->sweep.c; b->sweep.a0 = b->sweep.a;
        if (b->type == BT_DYNAMIC) {
            V2 g = vmul(b->gravityScale, w->gravity);
            V2 acc = vadd(g, vmul(b->invMass, b->force));
            v = vadd(v, vmul(h, acc));
            wv += h * b->invI * b->torque;
            { float s = 1.0f / (1.0f + h * b->linearDamping); v.x *= s; v.y *= s; }
            wv *= 1.0f / (1.0f + h * b->angularDamping);
        }
        is->positions[i].c = c; is->positions[i].a = a;
        is->velocities[i].v = v; is->velocities[i].w = wv;
    }
    Solver s;
    solver_init(&s, step, is->contacts, is->contactCount, is->positions, is->velocities);
    solver_init_velocity_constraints(&s);
    if (step.warmStarting) solver_warm_start(&s);
#ifdef OR_NO_WORK
    velocity_sweeps(&s, step.velocityIterations, is->bodyCount);
    solver_store_impulses(&s);
    integrate_positions(is, h, 0);
    for (int i = 0; i < step.positionIterations; ++i) {
        w->posIters++;
        if (solver_solve_position(&s, 0, -1, -1)) break;
    }
#else
    const int sweeps = work_velocity_sweeps(&s, step.velocityIterations, is->bodyCount);
    w->velIters += (long)step.velocityIterations * is->contactCount;
    solver_store_impulses(&s);
    integrate_positions(is, h, 0);
    int passes = 0;
    for (int i = 0; i < step.positionIterations; ++i) {
        w->posIters++;
        ++passes;
        if (solver_solve_position(&s, 0, -1, -1)) break;
    }
    if (g_topo_diag && g_topo_diag < 3 && is->contactCount >= (g_topo_diag > 1 ? 1 : 3) && is->contactCount <= 4) topo_record(&s, is, sweeps);
    if (g_topo_diag == 3 && is->contactCount >= 5 && sweeps >= 100) topo_print(&s, is, sweeps);
    if (is->contactCount > 0) {
        int dyn[256], lp = 0, pts = 0, n1 = 0, n2 = 0;
        for (int k = 0; k < is->bodyCount && k < 256; ++k) dyn[k] = is->bodies[k]->invMass > 0.0f || is->bodies[k]->invI > 0.0f;
        const int L = work_levels(&s, dyn, &lp);
        for (int i = 0; i < s.count; ++i) { pts += s.pcs[i].pointCount; if (s.vcs[i].pointCount == 2) ++n2; else ++n1; }
        OrWork* k = &w->work;
        k->islands += 1; k->vel_sweeps += sweeps;
        k->vel_upd1 += (long)sweeps * n1; k->vel_upd2 += (long)sweeps * n2; k->vel_levels += (long)sweeps * L;
        k->pos_passes += passes; k->pos_points += (long)passes * pts; k->pos_level_points += (long)passes * lp;
        k->vel_pipe += work_pipe(&s, dyn, sweeps, 0);
        k->pos_pipe += work_pipe(&s, dyn, passes, 1);
        work_model_2wave(&s, dyn, sweeps, step.velocityIterations, k);
        const long units = (long)sweeps * s.count + (long)passes * pts;
        k->isl_units += units;
        w->stepIslSum += units;
        if (units > w->stepIslMax) w->stepIslMax = units;
    }
#endif
    for (int i = 0; i < is->bodyCount; ++i) {
        Body* body = is->bodies[i];
        body->sweep.c = is->positions[i].c; body->sweep.a = is->positions[i].a;
        body->v = is->velocities[i].v; body->w = is->velocities[i].w;
        body_synchronize_transform(body);
    }
    solver_free(&s);
}

static void island_solve_toi(Island* is, TimeStep sub, int toiIndexA, int toiIndexB, OrWork* k) {
    for (int i = 0; i < is->bodyCount; ++i) {
        Body* b = is->bodies[i];
        is->positions[i].c = b->sweep.c; is->positions[i].a = b->sweep.a;
        is->velocities[i].v = b->v; is->velocities[i].w = b->w;
    }
    Solver s;
    solver_init(&s, sub, is->contacts, is->contactCount, is->positions, is->velocities);
#ifdef OR_NO_WORK
    (void)k;
    for (int i = 0; i < sub.positionIterations; ++i)
        if (solver_solve_position(&s, 1, toiIndexA, toiIndexB)) break;
    is->bodies[toiIndexA]->sweep.c0 = is->positions[toiIndexA].c;
    is->bodies[toiIndexA]->sweep.a0 = is->positions[toiIndexA].a;
    is->bodies[toiIndexB]->sweep.c0 = is->positions[toiIndexB].c;
    is->bodies[toiIndexB]->sweep.a0 = is->positions[toiIndexB].a;
    solver_init_velocity_constraints(&s);
    velocity_sweeps(&s, sub.velocityIterations, is->bodyCount);
#else
    int passes = 0;
    for (int i = 0; i < sub.positionIterations; ++i) {
        ++passes;
        if (solver_solve_position(&s, 1, toiIndexA, toiIndexB)) break;
    }
    {   /* work model: in the TOI position passes only the TOI pair moves */
        int dyn[256], lp = 0, pts = 0;
        for (int q = 0; q < is->bodyCount && q < 256; ++q) dyn[q] = q == toiIndexA || q == toiIndexB;
        work_levels(&s, dyn, &lp);
        for (int i = 0; i < s.count; ++i) pts += s.pcs[i].pointCount;
        k->toi_pos_points += (long)passes * pts; k->toi_pos_level_points += (long)passes * lp;
        k->pos_pipe += work_pipe(&s, dyn, passes, 1);
    }
    is->bodies[toiIndexA]->sweep.c0 = is->positions[toiIndexA].c;
    is->bodies[toiIndexA]->sweep.a0 = is->positions[toiIndexA].a;
    is->bodies[toiIndexB]->sweep.c0 = is->positions[toiIndexB].c;
    is->bodies[toiIndexB]->sweep.a0 = is->positions[toiIndexB].a;
    solver_init_velocity_constraints(&s);
    const int sweeps = work_velocity_sweeps(&s, sub.velocityIterations, is->bodyCount);
    {
        int dyn[256];
        for (int q = 0; q < is->bodyCount && q < 256; ++q) dyn[q] = is->bodies[q]->invMass > 0.0f || is->bodies[q]->invI > 0.0f;
        const int L = work_levels(&s, dyn, NULL);
        k->toi_vel_upd += (long)sweeps * s.count; k->toi_vel_levels += (long)sweeps * L;
        k->vel_pipe += work_pipe(&s, dyn, sweeps, 0);
    }
#endif
    integrate_positions(is, sub.dt, 1);
    solver_free(&s);
}

/* ---------------------------------------------------------------- GJK distance [B2 b2Distance.cpp] */
typedef struct { const V2* v; int count; float radius; } DProxy;
typedef struct { float metric; int count; int indexA[3], indexB[3]; } SimplexCache;
typedef struct { V2 wA, wB, w; float a; int indexA, indexB; } SVertex;
typedef struct { SVertex v[3]; int count; } Simplex;

static int proxy_support(const DProxy* p, V2 d) {
    int best = 0; float bestValue = vdot(p->v[0], d);
    for (int i = 1; i < p->count; ++i) {
        float value = vdot(p->v[i], d);
        if (value > bestValue) { best = i; bestValue = value; }
    }
    return best;
}
static float vdist(V2 a, V2 b) { return vlen(vsub(a, b)); }
static float simplex_metric(const Simplex* s) {
    switch (s->count) {
    case 1: return 0.0f;
    case 2: return vdist(s->v[0].w, s->v[1].w);
    case 3: return vcross(vsub(s->v[1].w, s->v[0].w), vsub(s->v[2].w, s->v[0].w));
    default: return 0.0f;
    }
}
static void simplex_read_cache(Simplex* s, const SimplexCache* cache, const DProxy* pA, Xf xA, const DProxy* pB, Xf xB) {
    s->count = cache->count;
    for (int i = 0; i < s->count; ++i) {
        SVertex* v = s->v + i;
        v->indexA = cache->indexA[i]; v->indexB = cache->indexB[i];
        v->wA = mul_xv(xA, pA->v[v->indexA]); v->wB = mul_xv(xB, pB->v[v->indexB]);
        v->w = vsub(v->wB, v->wA); v->a = 0.0f;
    }
    if (s->count > 1) {
        float metric1 = cache->metric, metric2 = simplex_metric(s);
        if (metric2 < 0.5f * metric1 || 2.0f * metric1 < metric2 || metric2 < FLT_EPSILON) s->count = 0;
    }
    if (s->count == 0) {
        SVertex* v = s->v;
        v->indexA = 0; v->indexB = 0;
        v->wA = mul_xv(xA, pA->v[0]); v->wB = mul_xv(xB, pB->v[0]);
        v->w = vsub(v->wB, v->wA); v->a = 1.0f; s->count = 1;
    }
}
static void simplex_write_cache(const Simplex* s, SimplexCache* cache) {
    cache->metric = simplex_metric(s);
    cache->count = s->count;
    for (int i = 0; i < s->count; ++i) { cache->indexA[i] = s->v[i].indexA; cache->indexB[i] = s->v[i].indexB; }
}
static V2 simplex_search_dir(const Simplex* s) {
    if (s->count == 1) return vneg(s->v[0].w);
    V2 e12 = vsub(s->v[1].w, s->v[0].w);
    float sgn = vcross(e12, vneg(s->v[0].w));
    if (sgn > 0.0f) return vcross_sv(1.0f, e12);
    return vcross_vs(e12, 1.0f);
}
static V2 simplex_closest(const Simplex* s) {
    switch (s->count) {
    case 1: return s->v[0].w;
    case 2: return vadd(vmul(s->v[0].a, s->v[0].w), vmul(s->v[1].a, s->v[1].w));
    default: return v2(0.0f, 0.0f);
    }
}
static void simplex_witness(const Simplex* s, V2* pA, V2* pB) {
    switch (s->count) {
    case 1: *pA = s->v[0].wA; *pB = s->v[0].wB; break;
    case 2:
        *pA = vadd(vmul(s->v[0].a, s->v[0].wA), vmul(s->v[1].a, s->v[1].wA));
        *pB = vadd(vmul(s->v[0].a, s->v[0].wB), vmul(s->v[1].a, s->v[1].wB));
        break;
    case 3:
        *pA = vadd(vadd(vmul(s->v[0].a, s->v[0].wA), vmul(s->v[1].a, s->v[1].wA)), vmul(s->v[2].a, s->v[2].wA));
        *pB = *pA;
        break;
    default: break;
    }
}
static void simplex_solve2(Simplex* s) {
    V2 w1 = s->v[0].w, w2 = s->v[1].w;
    V2 e12 = vsub(w2, w1);
    float d12_2 = -vdot(w1, e12);
    if (d12_2 <= 0.0f) { s->v[0].a = 1.0f; s->count = 1; return; }
    float d12_1 = vdot(w2, e12);
    if (d12_1 <= 0.0f) { s->v[1].a = 1.0f; s->count = 1; s->v[0] = s->v[1]; return; }
    float inv = 1.0f / (d12_1 + d12_2);
    s->v[0].a = d12_1 * inv; s->v[1].a = d12_2 * inv; s->count = 2;
}
static void simplex_solve3(Simplex* s) {
    V2 w1 = s->v[0].w, w2 = s->v[1].w, w3 = s->v[2].w;
    V2 e12 = vsub(w2, w1);
    float w1e12 = vdot(w1, e12), w2e12 = vdot(w2, e12);
    float d12_1 = w2e12, d12_2 = -w1e12;
    V2 e13 = vsub(w3, w1);
    float w1e13 = vdot(w1, e13), w3e13 = vdot(w3, e13);
    float d13_1 = w3e13, d13_2 = -w1e13;
    V2 e23 = vsub(w3, w2);
    float w2e23 = vdot(w2, e23), w3e23 = vdot(w3, e23);
    float d23_1 = w3e23, d23_2 = -w2e23;
    float n123 = vcross(e12, e13);
    float d123_1 = n123 * vcross(w2, w3);
    float d123_2 = n123 * vcross(w3, w1);
    float d123_3 = n123 * vcross(w1, w2);
    if (d12_2 <= 0.0f && d13_2 <= 0.0f) { s->v[0].a = 1.0f; s->count = 1; return; }
    if (d12_1 > 0.0f && d12_2 > 0.0f && d123_3 <= 0.0f) {
        float inv = 1.0f / (d12_1 + d12_2); s->v[0].a = d12_1 * inv; s->v[1].a = d12_2 * inv; s->count = 2; return;
    }
    if (d13_1 > 0.0f && d13_2 > 0.0f && d123_2 <= 0.0f) {
        float inv = 1.0f / (d13_1 + d13_2); s->v[0].a = d13_1 * inv; s->v[2].a = d13_2 * inv; s->count = 2; s->v[1] = s->v[2]; return;
    }
    if (d12_1 <= 0.0f && d23_2 <= 0.0f) { s->v[1].a = 1.0f; s->count = 1; s->v[0] = s->v[1]; return; }
    if (d13_1 <= 0.0f && d23_1 <= 0.0f) { s->v[2].a = 1.0f; s->count = 1; s->v[0] = s->v[2]; return; }
    if (d23_1 > 0.0f && d23_2 > 0.0f && d123_1 <= 0.0f) {
        float inv = 1.0f / (d23_1 + d23_2); s->v[1].a = d23_1 * inv; s->v[2].a = d23_2 * inv; s->count = 2; s->v[0] = s->v[2]; return;
    }
    float inv = 1.0f / (d123_1 + d123_2 + d123_3);
    s->v[0].a = d123_1 * inv; s->v[1].a = d123_2 * inv; s->v[2].a = d123_3 * inv; s->count = 3;
}

static float gjk_distance(SimplexCache* cache, const DProxy* pA, Xf xA, const DProxy* pB, Xf xB) {
    Simplex s;
    simplex_read_cache(&s, cache, pA, xA, pB, xB);
    int saveA[3], saveB[3], saveCount = 0;
    int iter = 0;
    while (iter < 20) {
        saveCount = s.count;
        for (int i = 0; i < saveCount; ++i) { saveA[i] = s.v[i].indexA; saveB[i] = s.v[i].indexB; }
        if (s.count == 2) simplex_solve2(&s);
        else if (s.count == 3) simplex_solve3(&s);
        if (s.count == 3) break;
        (void)simplex_closest(&s);
        V2 d = simplex_search_dir(&s);
        if (vlensq(d) < FLT_EPSILON * FLT_EPSILON) break;
        SVertex* vtx = s.v + s.count;
        vtx->indexA = proxy_support(pA, mulT_rv(xA.q, vneg(d)));
        vtx->wA = mul_xv(xA, pA->v[vtx->indexA]);
        vtx->indexB = proxy_support(pB, mulT_rv(xB.q, d));
        vtx->wB = mul_xv(xB, pB->v[vtx->indexB]);
        vtx->w = vsub(vtx->wB, vtx->wA);
        ++iter;
        int dup = 0;
        for (int i = 0; i < saveCount; ++i) if (vtx->indexA == saveA[i] && vtx->indexB == saveB[i]) { dup = 1; break; }
        if (dup) break;
        ++s.count;
    }
    V2 pa = v2(0.0f, 0.0f), pb = v2(0.0f, 0.0f);
    simplex_witness(&s, &pa, &pb);
    float distance = vdist(pa, pb);
    simplex_write_cache(&s, cache);
    return distance;
}

/* ---------------------------------------------------------------- TOI [B2 b2TimeOfImpact.cpp] */
enum { SF_POINTS = 0, SF_FACEA = 1, SF_FACEB = 2 };
typedef struct { const DProxy* pA; const DProxy* pB; Sweep sA, sB; int type; V2 localPoint, axis; } SepFn;

static float sep_init(SepFn* f, const SimplexCache* cache, const DProxy* pA, Sweep sA, const DProxy* pB, Sweep sB, float t1) {
    f->pA = pA; f->pB = pB; f->sA = sA; f->sB = sB;
    Xf xfA, xfB;
    sweep_get_transform(&f->sA, &xfA, t1);
    sweep_get_transform(&f->sB, &xfB, t1);
    if (cache->count == 1) {
        f->type = SF_POINTS;
        V2 pointA = mul_xv(xfA, pA->v[cache->indexA[0]]);
        V2 pointB = mul_xv(xfB, pB->v[cache->indexB[0]]);
        f->axis = vsub(pointB, pointA);
        return vnormalize(&f->axis);
    } else if (cache->indexA[0] == cache->indexA[1]) {
        f->type = SF_FACEB;
        V2 lB1 = pB->v[cache->indexB[0]], lB2 = pB->v[cache->indexB[1]];
        f->axis = vcross_vs(vsub(lB2, lB1), 1.0f);
        vnormalize(&f->axis);
        V2 normal = mul_rv(xfB.q, f->axis);
        f->localPoint = vmul(0.5f, vadd(lB1, lB2));
        V2 pointB = mul_xv(xfB, f->localPoint);
        V2 pointA = mul_xv(xfA, pA->v[cache->indexA[0]]);
        float s = vdot(vsub(pointA, pointB), normal);
        if (s < 0.0f) { f->axis = vneg(f->axis); s = -s; }
        return s;
    } else {
        f->type = SF_FACEA;
        V2 lA1 = pA->v[cache->indexA[0]], lA2 = pA->v[cache->indexA[1]];
        f->axis = vcross_vs(vsub(lA2, lA1), 1.0f);
        vnormalize(&f->axis);
        V2 normal = mul_rv(xfA.q, f->axis);
        f->localPoint = vmul(0.5f, vadd(lA1, lA2));
        V2 pointA = mul_xv(xfA, f->localPoint);
        V2 pointB = mul_xv(xfB, pB->v[cache->indexB[0]]);
        float s = vdot(vsub(pointB, pointA), normal);
        if (s < 0.0f) { f->axis = vneg(f->axis); s = -s; }
        return s;
    }
}
static float sep_find_min(const SepFn* f, int* indexA, int* indexB, float t) {
    Xf xfA, xfB;
    sweep_get_transform(&f->sA, &xfA, t);
    sweep_get_transform(&f->sB, &xfB, t);
    switch (f->type) {
    case SF_POINTS: {
        V2 axisA = mulT_rv(xfA.q, f->axis), axisB = mulT_rv(xfB.q, vneg(f->axis));
        *indexA = proxy_support(f->pA, axisA); *indexB = proxy_support(f->pB, axisB);
        V2 pointA = mul_xv(xfA, f->pA->v[*indexA]), pointB = mul_xv(xfB, f->pB->v[*indexB]);
        return vdot(vsub(pointB, pointA), f->axis);
    }
    case SF_FACEA: {
        V2 normal = mul_rv(xfA.q, f->axis);
        V2 pointA = mul_xv(xfA, f->localPoint);
        V2 axisB = mulT_rv(xfB.q, vneg(normal));
        *indexA = -1; *indexB = proxy_support(f->pB, axisB);
        V2 pointB = mul_xv(xfB, f->pB->v[*indexB]);
        return vdot(vsub(pointB, pointA), normal);
    }
    default: {
        V2 normal = mul_rv(xfB.q, f->axis);
        V2 pointB = mul_xv(xfB, f->localPoint);
        V2 axisA = mulT_rv(xfA.q, vneg(normal));
        *indexB = -1; *indexA = proxy_support(f->pA, axisA);
        V2 pointA = mul_xv(xfA, f->pA->v[*indexA]);
        return vdot(vsub(pointA, pointB), normal);
    }
    }
}
static float sep_eval(const SepFn* f, int indexA, int indexB, float t) {
    Xf xfA, xfB;
    sweep_get_transform(&f->sA, &xfA, t);
    sweep_get_transform(&f->sB, &xfB, t);
    switch (f->type) {
    case SF_POINTS: {
        V2 pointA = mul_xv(xfA, f->pA->v[indexA]), pointB = mul_xv(xfB, f->pB->v[indexB]);
        return vdot(vsub(pointB, pointA), f->axis);
    }
    case SF_FACEA: {
        V2 normal = mul_rv(xfA.q, f->axis);
        V2 pointA = mul_xv(xfA, f->localPoint);
        V2 pointB = mul_xv(xfB, f->pB->v[indexB]);
        return vdot(vsub(pointB, pointA), normal);
    }
    default: {
        V2 normal = mul_rv(xfB.q, f->axis);
        V2 pointB = mul_xv(xfB, f->localPoint);
        V2 pointA = mul_xv(xfA, f->pA->v[indexA]);
        return vdot(vsub(pointA, pointB), normal);
    }
    }
}

enum { TOI_UNKNOWN = 0, TOI_FAILED, TOI_OVERLAPPED, TOI_TOUCHING, TOI_SEPARATED };
static void time_of_impact(int* state_out, float* t_out, const DProxy* pA, const DProxy* pB, Sweep sweepA, Sweep sweepB, float tMax) {
    int state = TOI_UNKNOWN; float tout = tMax;
    sweep_normalize(&sweepA); sweep_normalize(&sweepB);
    float totalRadius = pA->radius + pB->radius;
    float target = fmax_(LINEAR_SLOP, totalRadius - 3.0f * LINEAR_SLOP);
    float tolerance = 0.25f * LINEAR_SLOP;
    float t1 = 0.0f;
    const int k_maxIterations = 20;
    int iter = 0;
    SimplexCache cache; cache.count = 0; cache.metric = 0.0f;
    for (;;) {
        Xf xfA, xfB;
        sweep_get_transform(&sweepA, &xfA, t1);
        sweep_get_transform(&sweepB, &xfB, t1);
        float distance = gjk_distance(&cache, pA, xfA, pB, xfB);
        if (distance <= 0.0f) { state = TOI_OVERLAPPED; tout = 0.0f; break; }
        if (distance < target + tolerance) { state = TOI_TOUCHING; tout = t1; break; }
        SepFn fcn;
        sep_init(&fcn, &cache, pA, sweepA, pB, sweepB, t1);
        int done = 0;
        float t2 = tMax;
        int pushBackIter = 0;
        for (;;) {
            int indexA, indexB;
            float s2 = sep_find_min(&fcn, &indexA, &indexB, t2);
            if (s2 > target + tolerance) { state = TOI_SEPARATED; tout = tMax; done = 1; break; }
            if (s2 > target - tolerance) { t1 = t2; break; }
            float s1 = sep_eval(&fcn, indexA, indexB, t1);
            if (s1 < target - tolerance) { state = TOI_FAILED; tout = t1; done = 1; break; }
            if (s1 <= target + tolerance) { state = TOI_TOUCHING; tout = t1; done = 1; break; }
            int rootIterCount = 0;
            float a1 = t1, a2 = t2;
            for (;;) {
                float t;
                if (rootIterCount & 1) t = a1 + (target - s1) * (a2 - a1) / (s2 - s1);
                else t = 0.5f * (a1 + a2);
                ++rootIterCount;
                float s = sep_eval(&fcn, indexA, indexB, t);
                if (fabsf(s - target) < tolerance) { t2 = t; break; }
                if (s > target) { a1 = t; s1 = s; } else { a2 = t; s2 = s; }
                if (rootIterCount == 50) break;
            }
            ++pushBackIter;
            if (pushBackIter == B2_MAX_POLY) break;
        }
        ++iter;
        if (done) break;
        if (iter == k_maxIterations) { state = TOI_FAILED; tout = t1; break; }
    }
    *state_out = state; *t_out = tout;
}

/* ---------------------------------------------------------------- world step [B2 b2World.cpp] */
static void world_solve(World* w, TimeStep step) {
    Island is;
    island_init(&is, w->bodyCount, w->cm.contactCount);
    for (Body* b = w->bodyList; b; b = b->next) b->flags &= ~BF_ISLAND;
    for (Contact* c = w->cm.contactList; c; c = c->next) c->flags &= ~CF_ISLAND;
    Body** stack = (Body**)calloc((size_t)(w->bodyCount + 1), sizeof(Body*));
    for (Body* seed = w->bodyList; seed; seed = seed->next) {
        if (seed->flags & BF_ISLAND) continue;
        if ((seed->flags & BF_AWAKE) == 0 || (seed->flags & BF_ACTIVE) == 0) continue;
        if (seed->type == BT_STATIC) continue;
        is.bodyCount = 0; is.contactCount = 0;
        int stackCount = 0;
        stack[stackCount++] = seed;
        seed->flags |= BF_ISLAND;
        while (stackCount > 0) {
            Body* b = stack[--stackCount];
            island_add_body(&is, b);
            b->flags |= BF_AWAKE;
            if (b->type == BT_STATIC) continue;
            for (ContactEdge* ce = b->contactList; ce; ce = ce->next) {
                Contact* contact = ce->contact;
                if (contact->flags & CF_ISLAND) continue;
                if ((contact->flags & CF_ENABLED) == 0 || (contact->flags & CF_TOUCHING) == 0) continue;
                island_add_contact(&is, contact);
                contact->flags |= CF_ISLAND;
                Body* other = ce->other;
                if (other->flags & BF_ISLAND) continue;
                stack[stackCount++] = other;
                other->flags |= BF_ISLAND;
            }
        }
        if (is.bodyCount > w->maxIslandBodies) w->maxIslandBodies = is.bodyCount;
        if (is.contactCount > w->maxIslandContacts) w->maxIslandContacts = is.contactCount;
        island_solve(&is, w, step);
        for (int i = 0; i < is.bodyCount; ++i) {
            Body* b = is.bodies[i];
            if (b->type == BT_STATIC) b->flags &= ~BF_ISLAND;
        }
    }
    free(stack);
    island_free(&is);
    for (Body* b = w->bodyList; b; b = b->next) {
        if ((b->flags & BF_ISLAND) == 0) continue;
        if (b->type == BT_STATIC) continue;
        body_synchronize_fixtures(b);
    }
    cm_find_new_contacts(&w->cm);
}

static void world_solve_toi(World* w, TimeStep step) {
    Island is;
    island_init(&is, 2 * MAX_TOI_CONTACTS, MAX_TOI_CONTACTS);
    if (w->stepComplete) {
        for (Body* b = w->bodyList; b; b = b->next) { b->flags &= ~BF_ISLAND; b->sweep.alpha0 = 0.0f; }
        for (Contact* c = w->cm.contactList; c; c = c->next) {
            c->flags &= ~(CF_TOI | CF_ISLAND); c->toiCount = 0; c->toi = 1.0f;
        }
    }
    for (;;) {
        Contact* minContact = NULL; float minAlpha = 1.0f;
        for (Contact* c = w->cm.contactList; c; c = c->next) {
            if ((c->flags & CF_ENABLED) == 0) continue;
            if (c->toiCount > MAX_SUBSTEPS) continue;
            float alpha = 1.0f;
            if (c->flags & CF_TOI) {
                alpha = c->toi;
            } else {
                Fixture* fA = c->fA; Fixture* fB = c->fB;
                Body* bA = fA->body; Body* bB = fB->body;
                int typeA = bA->type, typeB = bB->type;
                int activeA = (bA->flags & BF_AWAKE) && typeA != BT_STATIC;
                int activeB = (bB->flags & BF_AWAKE) && typeB != BT_STATIC;
                if (!activeA && !activeB) continue;
                int collideA = (bA->flags & BF_BULLET) || typeA != BT_DYNAMIC;
                int collideB = (bB->flags & BF_BULLET) || typeB != BT_DYNAMIC;
                if (!collideA && !collideB) continue;
                float alpha0 = bA->sweep.alpha0;
                if (bA->sweep.alpha0 < bB->sweep.alpha0) { alpha0 = bB->sweep.alpha0; sweep_advance(&bA->sweep, alpha0); }
                else if (bB->sweep.alpha0 < bA->sweep.alpha0) { alpha0 = bA->sweep.alpha0; sweep_advance(&bB->sweep, alpha0); }
                DProxy pA = { fA->shape.v, fA->shape.count, fA->shape.radius };
                DProxy pB = { fB->shape.v, fB->shape.count, fB->shape.radius };
                int state; float beta;
                time_of_impact(&state, &beta, &pA, &pB, bA->sweep, bB->sweep, 1.0f);
                w->work.toi_calls++;
                if (state == TOI_TOUCHING) alpha = fmin_(alpha0 + (1.0f - alpha0) * beta, 1.0f);
                else alpha = 1.0f;
                c->toi = alpha;
                c->flags |= CF_TOI;
            }
            if (alpha < minAlpha) { minContact = c; minAlpha = alpha; }
        }
        if (minContact == NULL || 1.0f - 10.0f * FLT_EPSILON < minAlpha) { w->stepComplete = 1; break; }
        w->toiEvents++;
        Fixture* fA = minContact->fA; Fixture* fB = minContact->fB;
        Body* bA = fA->body; Body* bB = fB->body;
        Sweep backup1 = bA->sweep, backup2 = bB->sweep;
        body_advance(bA, minAlpha);
        body_advance(bB, minAlpha);
        contact_update(minContact, &w->cm);
        minContact->flags &= ~CF_TOI;
        ++minContact->toiCount;
        if ((minContact->flags & CF_ENABLED) == 0 || (minContact->flags & CF_TOUCHING) == 0) {
            minContact->flags &= ~CF_ENABLED;
            bA->sweep = backup1; bB->sweep = backup2;
            body_synchronize_transform(bA); body_synchronize_transform(bB);
            continue;
        }
        bA->flags |= BF_AWAKE; bB->flags |= BF_AWAKE;
        is.bodyCount = 0; is.contactCount = 0;
        island_add_body(&is, bA); island_add_body(&is, bB); island_add_contact(&is, minContact);
        bA->flags |= BF_ISLAND; bB->flags |= BF_ISLAND; minContact->flags |= CF_ISLAND;
        Body* bodies[2] = { bA, bB };
        for (int i = 0; i < 2; ++i) {
            Body* body = bodies[i];
            if (body->type != BT_DYNAMIC) continue;
            for (ContactEdge* ce = body->contactList; ce; ce = ce->next) {
                if (is.bodyCount == is.bodyCapacity) break;
                if (is.contactCount == is.contactCapacity) break;
                Contact* contact = ce->contact;
                if (contact->flags & CF_ISLAND) continue;
                Body* other = ce->other;
                if (other->type == BT_DYNAMIC && (body->flags & BF_BULLET) == 0 && (other->flags & BF_BULLET) == 0) continue;
                Sweep backup = other->sweep;
                if ((other->flags & BF_ISLAND) == 0) body_advance(other, minAlpha);
                contact_update(contact, &w->cm);
                if ((contact->flags & CF_ENABLED) == 0) { other->sweep = backup; body_synchronize_transform(other); continue; }
                if ((contact->flags & CF_TOUCHING) == 0) { other->sweep = backup; body_synchronize_transform(other); continue; }
                contact->flags |= CF_ISLAND;
                island_add_contact(&is, contact);
                if (other->flags & BF_ISLAND) continue;
                other->flags |= BF_ISLAND;
                if (other->type != BT_STATIC) other->flags |= BF_AWAKE;
                island_add_body(&is, other);
            }
        }
        TimeStep sub;
        sub.dt = (1.0f - minAlpha) * step.dt;
        sub.inv_dt = 1.0f / sub.dt;
        sub.dtRatio = 1.0f;
        sub.positionIterations = 20;
        sub.velocityIterations = step.velocityIterations;
        sub.warmStarting = 0;
        if (is.bodyCount > w->maxToiIslandBodies) w->maxToiIslandBodies = is.bodyCount;
        if (is.contactCount > w->maxToiIslandContacts) w->maxToiIslandContacts = is.contactCount;
        island_solve_toi(&is, sub, bA->islandIndex, bB->islandIndex, &w->work);
        for (int i = 0; i < is.bodyCount; ++i) {
            Body* body = is.bodies[i];
            body->flags &= ~BF_ISLAND;
            if (body->type != BT_DYNAMIC) continue;
            body_synchronize_fixtures(body);
            for (ContactEdge* ce = body->contactList; ce; ce = ce->next) ce->contact->flags &= ~(CF_TOI | CF_ISLAND);
        }
        cm_find_new_contacts(&w->cm);
    }
    island_free(&is);
}

void b2o_step(World* w, float dt, int velIters, int posIters) {
    w->stepIslSum = 0; w->stepIslMax = 0;
    if (w->flags & WF_NEWFIXTURE) { cm_find_new_contacts(&w->cm); w->flags &= ~WF_NEWFIXTURE; }
    w->flags |= WF_LOCKED;
    TimeStep step;
    step.dt = dt; step.velocityIterations = velIters; step.positionIterations = posIters;
    step.inv_dt = dt > 0.0f ? 1.0f / dt : 0.0f;
    step.dtRatio = w->inv_dt0 * dt;
    step.warmStarting = 1;
    cm_collide(&w->cm);
    for (Contact* c = w->cm.contactList; c; c = c->next) w->touching += (c->flags & CF_TOUCHING) != 0;
    if (w->stepComplete && step.dt > 0.0f) world_solve(w, step);
    if (step.dt > 0.0f) world_solve_toi(w, step);
    if (step.dt > 0.0f) w->inv_dt0 = step.inv_dt;
    if (w->flags & WF_CLEARFORCES) {
        for (Body* b = w->bodyList; b; b = b->next) { b->force = v2(0.0f, 0.0f); b->torque = 0.0f; }
    }
    w->flags &= ~WF_LOCKED;
    w->work.isl_concurrent_save += w->stepIslSum - w->stepIslMax;
}
