// mrp_render.h -- batched rgb_array rendering of lanes straight from the SoA lane state
// (SURVEY.md section 8f-3).  Included by mrp_lane.h after g_table is declared
// (RenderArgs, RBLOCK and RPPT live in mrp_ops.h).
//
// Replaces the pyglet/OpenGL `render(mode='rgb_array')` of the reference:
//   v0 / Heavy-v0 : gym_puzzles/envs/multi_robot_puzzle_00.py:528-592
//   v2 family     : gym_puzzles/envs/multi_robot_puzzle_02.py:590-661 (_render_human_vision)
//   v3            : gym_puzzles/envs/core.py:421-459 (+ Block.draw blocks.py:135-152, Robot.draw
//                   robot.py:76-87)
// The reference rasterises through OpenGL, which cannot run here; this kernel keeps its
// scene (draw order, shapes, colours, sizes) and defines the rasteriser exactly: a pixel
// takes the colour of the LAST primitive in draw order that contains its centre.
//   pixel (row r from the top, column c) -> world ((c+0.5)*sx, (H-1-r+0.5)*sy), f32;
//   polygon: every edge cross(v1-v0, p-v0) >= 0 (CCW, edges inclusive), vertices b2Mul(xf, v);
//   circle: dx*dx+dy*dy <= r*r; ring (unfilled circle, linewidth px): rin^2 <= d^2 <= rout^2;
//   polyline of width w: the union of axis-aligned rectangles of half-width w/2 around it.
// Circles are exact discs (the reference draws 30/100-gons).  Colours are round(255*c).
// All f32 arithmetic is evaluated without FMA contraction, so oracle/render_ref.py
// reproduces every pixel bit-for-bit.
#pragma once

namespace mrpr {

using namespace mrp;

enum : int { P_POLY = 0, P_CIRCLE = 1, P_RING = 2, P_RECT = 3 };
constexpr int MAXPRIM = 64;
constexpr float BPAD = 1e-4f;   // >> f32 rounding of the exact tests at these coordinates (|x| < 22 m)

struct Prim {
    int type, nv;
    uint32_t rgb;
    float a, b, c, d;          // circle: cx, cy, r^2 ; ring: cx, cy, rin^2, rout^2 ; rect: xlo, ylo, xhi, yhi
    float bx0, by0, bx1, by1;  // conservative bounding box (padded by BPAD): culls before the exact test
    float vx[MAX_POLY], vy[MAX_POLY];
};

__device__ __forceinline__ uint32_t rgb8(int r, int g, int b) { return (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16); }

__device__ inline void xf_point(float px, float py, float s, float c, float vx, float vy, float& ox, float& oy) {
    #pragma clang fp contract(off)
    ox = (c * vx - s * vy) + px;   // b2Mul(b2Transform, b2Vec2)
    oy = (s * vx + c * vy) + py;
}

template <int ENV>
__device__ inline void add_poly(Prim* P, int& n, const EnvTables& T, int f, float px, float py, float s, float c, uint32_t rgb) {
    #pragma clang fp contract(off)
    if (n >= MAXPRIM) return;   // pool guard (the largest scene, 3 blocks, holds 46 primitives)
    Prim& q = P[n++];
    q.type = P_POLY; q.rgb = rgb; q.nv = T.shape[f].count;
    for (int i = 0; i < q.nv; ++i) xf_point(px, py, s, c, T.shape[f].v[i].x, T.shape[f].v[i].y, q.vx[i], q.vy[i]);
    q.bx0 = q.bx1 = q.vx[0]; q.by0 = q.by1 = q.vy[0];
    for (int i = 1; i < q.nv; ++i) {
        q.bx0 = fminf(q.bx0, q.vx[i]); q.bx1 = fmaxf(q.bx1, q.vx[i]);
        q.by0 = fminf(q.by0, q.vy[i]); q.by1 = fmaxf(q.by1, q.vy[i]);
    }
    q.bx0 -= BPAD; q.by0 -= BPAD; q.bx1 += BPAD; q.by1 += BPAD;
}
__device__ inline void add_circle(Prim* P, int& n, float x, float y, float r, uint32_t rgb) {
    #pragma clang fp contract(off)
    if (n >= MAXPRIM) return;
    Prim& q = P[n++];
    q.type = P_CIRCLE; q.rgb = rgb; q.a = x; q.b = y; q.c = r * r; q.nv = 0;
    q.bx0 = x - r - BPAD; q.bx1 = x + r + BPAD; q.by0 = y - r - BPAD; q.by1 = y + r + BPAD;
}
__device__ inline void add_rect(Prim* P, int& n, float xlo, float ylo, float xhi, float yhi, uint32_t rgb) {
    #pragma clang fp contract(off)
    if (n >= MAXPRIM) return;
    Prim& q = P[n++];
    q.type = P_RECT; q.rgb = rgb; q.a = xlo; q.b = ylo; q.c = xhi; q.d = yhi; q.nv = 0;
    q.bx0 = xlo; q.by0 = ylo; q.bx1 = xhi; q.by1 = yhi;
}

// Display list of one lane, in the reference's draw order.
template <int ENV>
__device__ int build_scene(const LaneState<ENV>& S, const EnvTables& T, const RenderArgs& A, Prim* P) {
    #pragma clang fp contract(off)
    using D = Dims<ENV>;
    constexpr int NB = D::NB, ND = D::NA + D::NB;
    const uint32_t white = rgb8(255, 255, 255), grey = rgb8(128, 128, 128), wall = rgb8(51, 51, 51), blue = rgb8(58, 153, 255);
    int n = 0;
    if (D::V == 0) {
        // boundary polyline (BORDER=1 m, linewidth 3, colour 0.2): :548-555
        const float h = 1.5f * A.lw_unit, W = 640.0f / 30.0f, H = 480.0f / 30.0f;
        add_rect(P, n, 1.0f - h, 1.0f - h, W - 1.0f + h, 1.0f + h, wall);
        add_rect(P, n, W - 1.0f - h, 1.0f - h, W - 1.0f + h, H - 1.0f + h, wall);
        add_rect(P, n, 1.0f - h, H - 1.0f - h, W - 1.0f + h, H - 1.0f + h, wall);
        add_rect(P, n, 1.0f - h, 1.0f - h, 1.0f + h, H - 1.0f + h, wall);
    } else if (D::V == 2) {
        // final points first (_render_human_vision :629-634): white dot, dark-grey ring (linewidth 5)
        for (int b = 0; b < NB; ++b) {
            float fx = (float)(S.goal[b][0] * A.goal_scale), fy = (float)(S.goal[b][1] * A.goal_scale);
            add_circle(P, n, fx, fy, 0.0075f, white);
            Prim& q = P[n++];
            const float h = 2.5f * A.lw_unit, ri = A.ring_r - h, ro = A.ring_r + h;
            q.type = P_RING; q.rgb = wall; q.a = fx; q.b = fy; q.c = ri * ri; q.d = ro * ro; q.nv = 0;
            q.bx0 = fx - ro - BPAD; q.bx1 = fx + ro + BPAD; q.by0 = fy - ro - BPAD; q.by1 = fy + ro + BPAD;
        }
    }
    // drawlist = boundary + blocks + agents (:409 / _02.py:440); body.fixtures is head-inserted
    // [B2 b2Body::CreateFixture], so each body's fixtures are drawn in reverse creation order.
    for (int b = ND; b < ND + 4; ++b)
        for (int k = T.body_nfix[b] - 1; k >= 0; --k) add_poly<ENV>(P, n, T, T.body_fix0[b] + k, T.wall_px[b - ND], T.wall_py[b - ND], 0.0f, 1.0f, wall);
    // v3: the boundary is its four wall polygons only; Block.draw / Robot.draw use the v0 sizes
    const float lg = D::V == 2 ? 0.015f : 0.16f, sm = D::V == 2 ? 0.0075f : 0.08f;
    for (int b = 0; b < NB; ++b) {
        for (int k = T.body_nfix[b] - 1; k >= 0; --k) add_poly<ENV>(P, n, T, T.body_fix0[b] + k, S.xpx[b], S.xpy[b], S.xs[b], S.xc[b], grey);
        add_circle(P, n, S.cx[b], S.cy[b], lg, white);
        for (int k = T.body_nfix[b] - 1; k >= 0; --k) {
            const ShapeDef& sh = T.shape[T.body_fix0[b] + k];
            for (int i = 0; i < sh.count; ++i) {   // blks_vertices (duplicates repaint the same disc)
                float x, y;
                xf_point(S.xpx[b], S.xpy[b], S.xs[b], S.xc[b], sh.v[i].x, sh.v[i].y, x, y);
                add_circle(P, n, x, y, sm, white);
            }
        }
    }
    for (int b = NB; b < ND; ++b) {
        for (int k = T.body_nfix[b] - 1; k >= 0; --k)   // v2 wheels (k>0) grey, hull white
            add_poly<ENV>(P, n, T, T.body_fix0[b] + k, S.xpx[b], S.xpy[b], S.xs[b], S.xc[b], k > 0 ? grey : white);
        add_circle(P, n, S.xpx[b], S.xpy[b], lg, grey);   // COLORS['i_block']
    }
    if (D::V != 2) {   // final point, EPSILON/SCALE, blue (:588-590; v3 core.py:456-457)
        float fx = (float)(S.goal[0][0] * A.goal_scale), fy = (float)(S.goal[0][1] * A.goal_scale);
        add_circle(P, n, fx, fy, 25.0f / 30.0f, blue);
    }
    return n;
}

__device__ inline bool hit(const Prim& q, float x, float y) {
    #pragma clang fp contract(off)
    if (x < q.bx0 || x > q.bx1 || y < q.by0 || y > q.by1) return false;
    switch (q.type) {
    case P_POLY: {
        for (int i = 0; i < q.nv; ++i) {
            int j = i + 1 == q.nv ? 0 : i + 1;
            float ex = q.vx[j] - q.vx[i], ey = q.vy[j] - q.vy[i];
            float dx = x - q.vx[i], dy = y - q.vy[i];
            if (ex * dy - ey * dx < 0.0f) return false;
        }
        return true;
    }
    case P_CIRCLE: { float dx = x - q.a, dy = y - q.b; return dx * dx + dy * dy <= q.c; }
    case P_RING: { float dx = x - q.a, dy = y - q.b, d2 = dx * dx + dy * dy; return d2 >= q.c && d2 <= q.d; }
    default: return x >= q.a && x <= q.c && y >= q.b && y <= q.d;
    }
}

// grid: (ceil(W*H / (RBLOCK*RPPT)), n_sel).  One workgroup builds its lane's display list in LDS
// (thread 0; <= 64 primitives), then every thread shades RPPT pixels (RBLOCK apart), each by walking the list from
// the top (the last primitive drawn) and stopping at the first hit.  Output rows are written
// as contiguous RGB bytes, so consecutive threads store consecutive 3-byte pixels.
template <int ENV>
__global__ __launch_bounds__(RBLOCK) void k_render(const uint32_t* __restrict__ state, const int32_t* __restrict__ lanes, int n_lanes,
                                                   int W, int H, RenderArgs A, uint8_t* __restrict__ out) {
    #pragma clang fp contract(off)
    __shared__ Prim P[MAXPRIM];
    __shared__ int np;
    const int sel = blockIdx.y;
    const int lane = lanes[sel];
    if (threadIdx.x == 0) {
        np = 0;
        if (lane >= 0 && lane < n_lanes) {
            const LaneState<ENV>& S = *reinterpret_cast<const LaneState<ENV>*>(state + (size_t)lane * lane_words<ENV>());
            np = build_scene<ENV>(S, g_table, A, P);
        }
    }
    __syncthreads();
    for (int k = 0; k < RPPT; ++k) {
        const int pix = (blockIdx.x * RPPT + k) * RBLOCK + threadIdx.x;
        if (pix >= W * H) return;
        const int r = pix / W, c = pix - r * W;
        const float x = ((float)c + 0.5f) * A.sx, y = ((float)(H - 1 - r) + 0.5f) * A.sy;
        uint32_t rgb = 0;   // background: black
        for (int i = np - 1; i >= 0; --i)
            if (hit(P[i], x, y)) { rgb = P[i].rgb; break; }
        uint8_t* o = out + ((size_t)sel * W * H + pix) * 3;
        o[0] = (uint8_t)(rgb & 255); o[1] = (uint8_t)((rgb >> 8) & 255); o[2] = (uint8_t)(rgb >> 16);
    }
}

template <int ENV>
__global__ void k_goals(const uint32_t* __restrict__ state, int nl, double* out) {
    using D = Dims<ENV>;
    const int lane = blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= nl) return;
    const LaneState<ENV>& S = *reinterpret_cast<const LaneState<ENV>*>(state + (size_t)lane * lane_words<ENV>());
    for (int b = 0; b < D::NB; ++b)
        for (int k = 0; k < 3; ++k) out[((size_t)lane * D::NB + b) * 3 + k] = S.goal[b][k];
}

}  // namespace mrpr
