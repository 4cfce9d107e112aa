// mrt_device.hpp - device-side scene view, BVH traversal and primitive tests for gfx950.
//
// Reachability and tie semantics follow SURVEY.md Appendix A.7:
//   * a primitive is tested only if every ancestor box passes the reference slab predicate
//     (AABB.cpp:34-54, reproduced with libstdc++ min/max operand order);
//   * the closest hit is the lexicographic minimum of (t, kind, BVH index), which equals the
//     reference's "first visited wins on equal t" because its left-first DFS visits leaves in
//     ascending BVH primitive index (BVH.hpp:252-268, 357-373) and kinds in the order
//     planes, spheres, triangles, lights (Shader.cpp:104-111);
//   * traverse<> visits exactly the reference's set of boxes (no t-culling): it serves the tiny
//     plane / sphere BVHs and the per-wave reference walk; the persistent walk of
//     mrt_trace_ww.hpp culls triangle boxes with a rigorous bound (cullKey).
#pragma once

#include "mrt_common.hpp"

namespace mrt {

constexpr int kBlock = 256;         // threads per workgroup for every trace kernel
constexpr int kLdsStackMin = 8;     // per-thread stack entries (8 bytes) in LDS; deeper ones spill
static_assert((kLdsStackMin & (kLdsStackMin - 1)) == 0, "the LDS stack rings are indexed by a power-of-two mask");

struct DScene {
    const float4* triGeom;     // 3 per triangle (BVH order): A, AB, AC  (xyz)
    const float4* triShade;    // 3 per triangle: nA (w = material index bits), nB, nC
    const float4* triHead;     // 1 per triangle: nA, w = bits of ((material + 1) << 1 | flat): flat when
                               // nA, nB and nC are the same bits (then triShade is not read)
    const GNode* triNodes;     // the reference tree (triRootRef)
    const QNode4* triQNodes;   // the walk tree (triRoot), 4-wide and quantized (QNode4)
    // the same nodes for the packet walk's scalar loads (mrt_trace_packet.hpp), 128 B each: the 24
    // grid indices as floats (child c: min xyz, max xyz at [6c, 6c + 6)), then the 4 references
    const float* triQNodesF;
    // per leaf, indexed by its first triangle t (48 B): [3t] = min xyz, max x; [3t+1].xy = max yz
    // (walk-tree leaves are tested exactly before their triangles); [3t+1].zw, [3t+2] = the leaf's
    // certified-cull record (mrt_scene.cpp leafCullRecord; the exact cull mode)
    const float4* leafBoxes;
    const float4* planes;      // 2 per plane: normal (w = material bits), point
    const GNode* planeNodes;
    const float4* spheres;     // 2 per sphere: center (w = sqRadius), (x = material bits)
    const GNode* sphereNodes;
    const float4* lights;      // 4 per light: A or position (w = kind bits), AB, AC, Le
    const float4* mats;        // 4 per material: Le (w = ior), Kd, Ks, Kt
    // 2^20 x {shader (Shader.cpp:23), sampler (StaticHaltonSeq.cpp) shuffled Halton values,
    // cos and sin of 2 pi * shader entry by the host libm (fillHemisphereTrig)}
    const float4* tables;
    // per 8-entry block b, the values a shading vertex draws with samplesLight 1 (purposes 0-5):
    // [2b] = {sampler[8b] (Russian roulette), cos, sin of 2 pi shader[8b+1] (hemisphere r1),
    // shader[8b+2] (hemisphere r2)}, [2b+1] = {shader[8b+3] (light pick), sampler[8b+4],
    // sampler[8b+5] (area-light point), 0}: 32 B per vertex instead of a 128-B line, and a 4 MB
    // table instead of 16 MB (the same values, relocated)
    const float4* vertexDraws;
    const float2* jitterDraws;  // per block: the pixel sampler's two draws (tree code 0, RaygenArgs::jitter)
    // triRoot: the walk tree (the reference leaves regrouped, rebuildOverLeaves, quantized);
    // triRootRef: the reference tree (BVH.hpp) - for rays outside the quantized grid's error bound
    // (a non-finite or extreme 1/d, whose slab NaNs or roundings break the leaf-box reachability
    // argument), for the certified cull and for the per-wave reference walk
    GRoot triRoot, triRootRef, planeRoot, sphereRoot;
    QGrid qgrid;               // the walk tree's quantization grid
    int32_t qEnabled;          // 0: every ray walks the reference tree (a non-finite scene box)
    int32_t nLights;
    int32_t nMats;
    int32_t cull;              // walk 1's cull mode: 0 none, 1 fast, 2 certified, 3 exact (mrt_trace_ww.hpp)
    int32_t variant;           // trace walk: 0 per-wave reference walk, 1 persistent while-while
    int32_t triTop;            // triQNodes[0, triTop) are the breadth-first top of the walk tree
    int32_t matsFinite;        // every material's Kd / Ks / Kt component is finite
    int32_t anyOrder;          // shadow walk child order (tuning key 5): 0 near first, 1 far first (default)
    int32_t tailDonate;        // idle lanes of a level's tail help walking lanes (tuning key 8, mrt_trace_ww.hpp)
    int32_t refill;            // idle lanes before a walk wave fetches new rays (tuning key 9, default 32)
    int32_t leanShade;         // k_shade's lean instantiation where it applies (tuning key 10)
    int32_t packet;            // level-1 rays take the wave-coherent walk (tuning key 16; modes 0 / 3)
    int32_t fuseShade;         // level 1: the packet walk shades its own hits (set per pass: tuning key 17)
    // textures (map_Kd): scenes with a textured material only (`textured` != 0)
    const float4* triTex;      // 2 per triangle: (tA.xy, tB.xy), (tC.xy, -, -)
    const int4* texInfo;       // per texture: width, height, channels, first byte in texels
    const uint8_t* texels;
    int32_t textured;
    // Config::accelerator (Shader.hpp:20-24): 1 Naive, 2 RegularGrid, 3 BVH, anything else
    // builds no accelerator (only lights are hit, Shader.cpp:86-111)
    int32_t accel;
    const int* triNaive;       // Naive: BVH-order index of the i-th triangle / plane / sphere of the input
    const int* planeNaive;
    const int* sphereNaive;
    GGrid planeGrid, sphereGrid, triGrid;  // RegularGrid (accelerator 2 only)
};

__device__ __forceinline__ float4 ld4(const float4* p) { return *p; }
__device__ __forceinline__ v3 xyz(float4 a) { return v3{a.x, a.y, a.z}; }
__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __uint_as_float(u); }

// AABB.cpp:34-54 with the ray's reciprocal direction precomputed (same value: 1.0F / d[axis]).
// Returns the reference predicate; *tEntry = max(tMin, 0) for ordering / culling.
__device__ __forceinline__ bool slab(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, v3 o, v3 inv,
                                     float* tEntry) {
    const float t1x = (mnx - o.x) * inv.x;
    const float t2x = (mxx - o.x) * inv.x;
    float tMin = stdmin(t1x, t2x);
    float tMax = stdmax(t1x, t2x);
    const float t1y = (mny - o.y) * inv.y;
    const float t2y = (mxy - o.y) * inv.y;
    tMin = stdmax(tMin, stdmin(t1y, t2y));
    tMax = stdmin(tMax, stdmax(t1y, t2y));
    const float t1z = (mnz - o.z) * inv.z;
    const float t2z = (mxz - o.z) * inv.z;
    tMin = stdmax(tMin, stdmin(t1z, t2z));
    tMax = stdmin(tMax, stdmax(t1z, t2z));
    const float e = stdmax(tMin, 0.0F);
    *tEntry = e;
    return tMax >= e;
}

// The same predicate for rays whose 1/d components are all finite.  Then no operand can be
// NaN ((box - o) * finite is finite or +-inf), so IEEE min/max (v_min3 / v_max3) return the
// ternaries' values, up to the sign of a zero, which no comparison made with tEntry can see.
__device__ __forceinline__ bool slabFinite(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, v3 o,
                                           v3 inv, float* tEntry) {
    const float t1x = (mnx - o.x) * inv.x;
    const float t2x = (mxx - o.x) * inv.x;
    const float t1y = (mny - o.y) * inv.y;
    const float t2y = (mxy - o.y) * inv.y;
    const float t1z = (mnz - o.z) * inv.z;
    const float t2z = (mxz - o.z) * inv.z;
    const float e = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fmaxf(fminf(t1z, t2z), 0.0F));
    const float tMax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
    *tEntry = e;
    return tMax >= e;
}

// slabFinite that also returns each axis's entry t (min of the two plane crossings): the
// cull key inflates the box per axis (mrt_trace_ww.hpp cullKey).
__device__ __forceinline__ bool slabFiniteAxes(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, v3 o,
                                               v3 inv, float* tEntry, float* ex, float* ey, float* ez) {
    const float t1x = (mnx - o.x) * inv.x;
    const float t2x = (mxx - o.x) * inv.x;
    const float t1y = (mny - o.y) * inv.y;
    const float t2y = (mxy - o.y) * inv.y;
    const float t1z = (mnz - o.z) * inv.z;
    const float t2z = (mxz - o.z) * inv.z;
    *ex = fminf(t1x, t2x);
    *ey = fminf(t1y, t2y);
    *ez = fminf(t1z, t2z);
    const float e = fmaxf(fmaxf(*ex, *ey), fmaxf(*ez, 0.0F));
    const float tMax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
    *tEntry = e;
    return tMax >= e;
}

__device__ __forceinline__ bool finiteInv(v3 inv) {
    return __builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z);
}

// Short traversal stack of the cull modes: each entry is a child's reference and its entry t
// (8 B; culled entries are skipped at the pop).  The top `depth` (power of two) entries live in
// LDS (conflict-free layout [slot][thread]), deeper entries spill to a per-thread global area.
struct TStack {
    static constexpr bool kKeys = true;
    int2* lds;    // &ldsBase[threadIdx.x]; slot s at lds[s * stride]
    int2* gbase;  // overflow areas (kernel-uniform base) ...
    int gofs;     // ... and this thread's offset into them (32-bit: one VGPR)
    int sp;
    int depth;
    int stride;   // threads per workgroup
    __device__ __forceinline__ void push(int ref, float t) {
        const int slot = sp & (depth - 1);
        if (sp >= depth) gbase[gofs + sp - depth] = lds[slot * stride];
        lds[slot * stride] = make_int2(ref, __float_as_int(t));
        ++sp;
    }
    __device__ __forceinline__ int2 pop() {
        --sp;
        const int slot = sp & (depth - 1);
        const int2 v = lds[slot * stride];
        if (sp >= depth) lds[slot * stride] = gbase[gofs + sp - depth];
        return v;
    }
};

// The stack of the modes that never cull an inner node (0 and 3, the default): references only
// (4 B), so the same LDS holds twice the entries (16 per thread, [slot][thread]); deeper entries
// spill to the per-thread global area as TStack's do.
template <int kThreads>
struct RefStack {
    static constexpr bool kKeys = false;
    static constexpr int kDepth = 2 * kLdsStackMin;
    int* lds;    // &ldsBase[threadIdx.x]
    int* gbase;  // overflow areas ...
    int gofs;    // ... and this thread's offset into them
    int sp;
    __device__ __forceinline__ void push(int ref, float) {
        const int slot = sp & (kDepth - 1);
        if (sp >= kDepth) gbase[gofs + sp - kDepth] = lds[slot * kThreads];
        lds[slot * kThreads] = ref;
        ++sp;
    }
    __device__ __forceinline__ int2 pop() {  // (reference, 0)
        --sp;
        const int slot = sp & (kDepth - 1);
        const int v = lds[slot * kThreads];
        if (sp >= kDepth) lds[slot * kThreads] = gbase[gofs + sp - kDepth];
        return make_int2(v, 0);
    }
};

// A walk kernel's stack over its LDS array (kLdsStackMin int2 per thread) and its global spill
// area (gdepth int2 per thread, gdepth >= the tree's stack need - kLdsStackMin).
template <int kThreads>
__device__ __forceinline__ TStack makeKeyStack(int2* ldsBase, int2* gstack, int gdepth) {
    return TStack{ldsBase + threadIdx.x, gstack, static_cast<int>(blockIdx.x * kThreads + threadIdx.x) * gdepth, 0,
                  kLdsStackMin, kThreads};
}
template <int kThreads>
__device__ __forceinline__ RefStack<kThreads> makeRefStack(int2* ldsBase, int2* gstack, int gdepth) {
    return RefStack<kThreads>{reinterpret_cast<int*>(ldsBase) + threadIdx.x, reinterpret_cast<int*>(gstack),
                              static_cast<int>(blockIdx.x * kThreads + threadIdx.x) * gdepth * 2, 0};
}

struct Best {
    float t, u, v;
    uint32_t code;  // encodePrim(kind, index) or kNoPrim
};

// Triangle.cpp:63-109 (without the hit-record construction); returns t, u, v.
__device__ __forceinline__ bool triTest(float4 a4, float4 ab4, float4 ac4, v3 o, v3 d, float* tOut, float* uOut,
                                        float* vOut) {
    const v3 A = xyz(a4), AB = xyz(ab4), AC = xyz(ac4);
    const v3 p = cross(d, AC);
    const float det = dot(AB, p);
    if (fabsf(det) < kEpsilon) return false;
    const float inv = 1.0F / det;
    const v3 s = o - A;
    const float u = inv * dot(s, p);
    if (u < 0.0F || u > 1.0F) return false;
    const v3 q = cross(s, AB);
    const float v = inv * dot(d, q);
    if (v < 0.0F || (u + v) > 1.0F) return false;
    *tOut = inv * dot(AC, q);
    *uOut = u;
    *vOut = v;
    return true;
}

// lexicographic (t, kind, index) acceptance; `same` = candidate kind equals best kind
__device__ __forceinline__ bool betterThan(float t, uint32_t code, float bt, uint32_t bcode) {
    return !(t >= bt) || (t == bt && primKind(bcode) == primKind(code) && primIndex(code) < primIndex(bcode));
}
__device__ __forceinline__ bool better(float t, uint32_t code, const Best& b) { return betterThan(t, code, b.t, b.code); }

// kTies: the BVH walks' total order (equal t: lower index); false: Naive's plain `<` in input order
template <bool kAny, bool kTies = true>
__device__ __forceinline__ bool leafTriangles(const DScene& s, int first, int count, v3 o, v3 d, uint32_t src,
                                              Best* b, uint32_t* nTri) {
    for (int k = 0; k < count; ++k) {
        const int j = first + k;
        const uint32_t code = encodePrim(kTriangle, static_cast<uint32_t>(j));
        if (code == src) continue;  // Triangle.cpp:64-66 self-exclusion
        const float4* g = s.triGeom + 3 * j;
        float t, u, v;
        ++*nTri;
        if (!triTest(ld4(g), ld4(g + 1), ld4(g + 2), o, d, &t, &u, &v)) continue;
        if (t < kEpsilon) continue;
        if (kAny) {
            if (!(t >= b->t)) return true;
        } else if (kTies ? better(t, code, *b) : !(t >= b->t)) {
            b->t = t;
            b->u = u;
            b->v = v;
            b->code = code;
        }
    }
    return false;
}

// kTies: the BVH walks' total order (equal t: lower index); false: Naive's plain `<` in input order
template <bool kAny, bool kTies = true>
__device__ __forceinline__ bool leafPlanes(const DScene& s, int first, int count, v3 o, v3 d, uint32_t src, Best* b) {
    for (int k = 0; k < count; ++k) {  // Plane.cpp:38-72
        const int j = first + k;
        const uint32_t code = encodePrim(kPlane, static_cast<uint32_t>(j));
        if (code == src) continue;
        const v3 n = xyz(s.planes[2 * j]);
        const v3 p0 = xyz(s.planes[2 * j + 1]);
        const float den = dot(n, d);
        if (fabsf(den) < kEpsilon) continue;
        const v3 vtp = p0 - o;
        const float num = dot(n, vtp);
        const float t = num / den;
        if (t < kEpsilon) continue;
        if (kAny) {
            if (!(t >= b->t)) return true;
        } else if (kTies ? better(t, code, *b) : !(t >= b->t)) {
            b->t = t;
            b->u = 0.0F;
            b->v = 0.0F;
            b->code = code;
        }
    }
    return false;
}

template <bool kAny, bool kTies = true>
__device__ __forceinline__ bool leafSpheres(const DScene& s, int first, int count, v3 o, v3 d, Best* b) {
    for (int k = 0; k < count; ++k) {  // Sphere.cpp:42-81 (no self-exclusion)
        const int j = first + k;
        const float4 c4 = s.spheres[2 * j];
        const v3 oc = xyz(c4) - o;
        const float proj = dot(oc, d);
        const float ocMag = length(oc);
        const float a = dot(d, d);
        const float bq = 2.0F * -proj;
        const float c = ocMag * ocMag - c4.w;
        const float disc = bq * bq - 4.0F * a * c;
        if (disc < 0.0F) continue;
        const float r = sqrtf(disc);
        const float d1 = -bq + r;
        const float d2 = -bq - r;
        const float t = stdmin(d1, d2) / (2.0F * a);
        if (t < kEpsilonLarge) continue;
        const uint32_t code = encodePrim(kSphere, static_cast<uint32_t>(j));
        if (kAny) {
            if (!(t >= b->t)) return true;
        } else if (kTies ? better(t, code, *b) : !(t >= b->t)) {
            b->t = t;
            b->u = 0.0F;
            b->v = 0.0F;
            b->code = code;
        }
    }
    return false;
}

struct TravCount {
    uint32_t nodes;  // child records fetched (2 per inner visit)
    uint32_t tris;   // triangle tests
    uint32_t leaves = 0;    // leaf records fetched (the walk tree's exact leaf boxes)
    uint32_t rayStart = 0;  // nodes at the current ray's fetch (per-ray maximum, counting builds)
    uint32_t rayMax = 0;
    uint32_t rays = 0;      // rays this lane fetched (the wave log of counting builds)
    uint32_t occluded = 0;  // any hit: occluded rays
    // walk phases (wave iterations counted once per wave, by its first active lane): inner-node
    // visits, leaf tests, triangle tests, and the lanes active in them
    uint32_t innerIters = 0, innerLanes = 0, leafIters = 0, leafLanes = 0, triIters = 0, triLanes = 0;
    uint32_t innerIdle = 0, innerDone = 0;  // per inner iteration: lanes without a ray / with a finished one
};

// Generic BVH walk.  kKind selects the leaf routine.  Returns true on an any-hit.
// Naive::intersect (Naive.hpp): every primitive in input order, planes, spheres, triangles
// (Shader.cpp:90-94), each test rejecting t >= the current best (so ties go to the earlier
// primitive); a shadow ray returns at its first hit closer than its distance.  No boxes.
template <bool kAny>
__device__ __forceinline__ bool naiveWalk(const DScene& s, v3 o, v3 d, uint32_t src, Best* b) {
    uint32_t nTri = 0;
    for (int i = 0; i < s.planeRoot.count; ++i)
        if (leafPlanes<kAny, false>(s, s.planeNaive[i], 1, o, d, src, b)) return true;
    for (int i = 0; i < s.sphereRoot.count; ++i)
        if (leafSpheres<kAny, false>(s, s.sphereNaive[i], 1, o, d, b)) return true;
    for (int i = 0; i < s.triRoot.count; ++i)
        if (leafTriangles<kAny, false>(s, s.triNaive[i], 1, o, d, src, b, &nTri)) return true;
    return false;
}

// RegularGrid<T>::intersect (RegularGrid.hpp:333-515): the 3D-DDA from the origin's (clamped)
// cell.  Every primitive of a visited cell is tested in list order with the plain `t >= best`
// rejection (ties: the first tested wins; a primitive listed in several cells is re-tested with
// the same result).  Shadow rays return at the first primitive closer than their distance.  A
// closest-hit walk stops at the grid's edge or, once THIS kind has improved the hit (the jump to
// `testloop`), at the first cell boundary beyond the hit.  Every step moves one axis toward its
// exit, so at most 3 x kGridSize cells are visited.
template <int kKind, bool kAny>
__device__ __forceinline__ bool gridWalk(const DScene& s, const GGrid& g, v3 o, v3 d, uint32_t src, Best* b) {
    if (g.count == 0) return false;  // no primitive of this kind: nothing is ever tested
    const v3 mn{g.mn[0], g.mn[1], g.mn[2]}, cs{g.cs[0], g.cs[1], g.cs[2]};
    // RegularGrid.hpp:337-347
    int c[3];
    const float cf[3] = {(o.x - mn.x) * g.csi[0], (o.y - mn.y) * g.csi[1], (o.z - mn.z) * g.csi[2]};
    int step[3], out[3];
    float tmax[3], tdelta[3] = {0.0F, 0.0F, 0.0F};
    const float dir[3] = {d.x, d.y, d.z}, org[3] = {o.x, o.y, o.z}, mnA[3] = {mn.x, mn.y, mn.z}, csA[3] = {cs.x, cs.y, cs.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        int ci = x86Trunc(cf[a]);
        ci = min(ci, kGridSize - 1);
        ci = max(ci, 0);
        c[a] = ci;
        float cb;  // RegularGrid.hpp:353-381
        if (dir[a] > 0) {
            step[a] = 1;
            out[a] = kGridSize;
            cb = mnA[a] + (static_cast<float>(ci) + 1.0F) * csA[a];
        } else {
            step[a] = -1;
            out[a] = -1;
            cb = mnA[a] + static_cast<float>(ci) * csA[a];
        }
        if (fabsf(dir[a]) > 1.19209290e-07F) {  // numeric_limits<float>::epsilon(), :384-406
            const float r = 1.0F / dir[a];
            tmax[a] = (cb - org[a]) * r;
            tdelta[a] = csA[a] * static_cast<float>(step[a]) * r;
        } else {
            tmax[a] = kRayLengthMax;
        }
    }
    bool improved = false;  // this kind has found a closer hit (the reference's jump to testloop)
    for (int iter = 0; iter <= 3 * kGridSize; ++iter) {
        const int cell = c[0] + (c[1] << kGridShift) + (c[2] << (2 * kGridShift));
        const int e = g.start[cell + 1];
        uint32_t nTri = 0;
        for (int k = g.start[cell]; k < e; ++k) {
            const int j = g.items[k];
            const float before = b->t;
            bool any = false;
            if (kKind == kTriangle) any = leafTriangles<kAny, false>(s, j, 1, o, d, src, b, &nTri);
            if (kKind == kPlane) any = leafPlanes<kAny, false>(s, j, 1, o, d, src, b);
            if (kKind == kSphere) any = leafSpheres<kAny, false>(s, j, 1, o, d, b);
            if (kAny && any) return true;
            improved = improved || b->t < before;
        }
        // RegularGrid.hpp:429-457 / 472-512
        const int a = tmax[0] < tmax[1] ? (tmax[0] < tmax[2] ? 0 : 2) : (tmax[1] < tmax[2] ? 1 : 2);
        const float tm = a == 0 ? tmax[0] : (a == 1 ? tmax[1] : tmax[2]);
        if (improved && b->t < tm) break;
        c[a] += step[a];
        if (c[a] == out[a]) break;
        const float td = a == 0 ? tdelta[0] : (a == 1 ? tdelta[1] : tdelta[2]);
        if (a == 0) tmax[0] = tm + td;
        else if (a == 1) tmax[1] = tm + td;
        else tmax[2] = tm + td;
    }
    return false;
}

template <int kKind, bool kAny, class Stack>
__device__ __forceinline__ bool traverse(const DScene& s, const GNode* nodes, const GRoot& root, v3 o, v3 d, v3 inv,
                                         uint32_t src, Best* b, Stack& st, TravCount* cnt) {
    if (root.count == 0) return false;  // BVH.hpp:328-330
    float te;
    if (!slab(root.bmin[0], root.bmin[1], root.bmin[2], root.bmax[0], root.bmax[1], root.bmax[2], o, inv, &te))
        return false;
    const int base = st.sp;
    int ref = root.ref;
    while (true) {
        if (ref >= 0) {
            const float4* np = reinterpret_cast<const float4*>(nodes + ref);
            const float4 n0 = np[0], n1 = np[1], n2 = np[2];
            const int4 n3 = reinterpret_cast<const int4*>(np)[3];
            cnt->nodes += 2;
            float tl, tr;
            const bool hl = slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, o, inv, &tl);
            const bool hr = slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, o, inv, &tr);
            if (hl && hr) {  // BVH.hpp:357-373: left first, right pushed
                st.push(n3.y, tr);
                ref = n3.x;
                continue;
            }
            if (hl) {
                ref = n3.x;
                continue;
            }
            if (hr) {
                ref = n3.y;
                continue;
            }
        } else {
            const int first = leafFirst(ref), count = leafCount(ref);
            bool any = false;
            if (kKind == kTriangle) any = leafTriangles<kAny>(s, first, count, o, d, src, b, &cnt->tris);
            if (kKind == kPlane) any = leafPlanes<kAny>(s, first, count, o, d, src, b);
            if (kKind == kSphere) any = leafSpheres<kAny>(s, first, count, o, d, b);
            if (kAny && any) {
                st.sp = base;
                return true;
            }
        }
        if (st.sp == base) return false;
        ref = st.pop().x;
    }
}

// Shader::rayTrace intersection part (Shader.cpp:86-111): planes, spheres, triangles, lights.
template <class Stack>
__device__ __forceinline__ Best closestHit(const DScene& s, v3 o, v3 d, uint32_t src, Stack& st, TravCount* cnt) {
    const v3 inv = v3{1.0F / d.x, 1.0F / d.y, 1.0F / d.z};
    Best b{kRayLengthMax, 0.0F, 0.0F, kNoPrim};
    traverse<kPlane, false>(s, s.planeNodes, s.planeRoot, o, d, inv, src, &b, st, cnt);
    traverse<kSphere, false>(s, s.sphereNodes, s.sphereRoot, o, d, inv, src, &b, st, cnt);
    traverse<kTriangle, false>(s, s.triNodes, s.triRootRef, o, d, inv, src, &b, st, cnt);
    for (int j = 0; j < s.nLights; ++j) {  // Shader.cpp:166-171, AreaLight.cpp:32-41
        const float4* l = s.lights + 4 * j;
        const float4 a4 = l[0];
        if (__float_as_int(a4.w) != 1) continue;  // point lights are never hit
        float t, u, v;
        if (!triTest(a4, l[1], l[2], o, d, &t, &u, &v)) continue;
        if (t < kEpsilon) continue;
        const uint32_t code = encodePrim(kLight, static_cast<uint32_t>(j));
        if (better(t, code, b)) {
            b.t = t;
            b.u = u;
            b.v = v;
            b.code = code;
        }
    }
    return b;
}

// Shader::shadowTrace (Shader.cpp:132-158): any hit closer than `dist`, lights excluded.
template <class Stack>
__device__ __forceinline__ bool anyHit(const DScene& s, v3 o, v3 d, uint32_t src, float dist, Stack& st,
                                       TravCount* cnt) {
    const v3 inv = v3{1.0F / d.x, 1.0F / d.y, 1.0F / d.z};
    Best b{dist, 0.0F, 0.0F, kNoPrim};
    if (traverse<kPlane, true>(s, s.planeNodes, s.planeRoot, o, d, inv, src, &b, st, cnt)) return true;
    if (traverse<kSphere, true>(s, s.sphereNodes, s.sphereRoot, o, d, inv, src, &b, st, cnt)) return true;
    return traverse<kTriangle, true>(s, s.triNodes, s.triRootRef, o, d, inv, src, &b, st, cnt);
}

}  // namespace mrt
