// mrt_trace_ww.hpp - persistent "while-while" triangle-BVH traversal for wave64.
//
// Same reachability, culling and tie rules as traverse<> in mrt_device.hpp (so results are
// identical, tested), organised for SIMD efficiency on CDNA's 64-lane waves:
//   * the walk tree is the reference's leaves regrouped and collapsed to a quantized 4-wide tree
//     (QNode4: 16-bit grid boxes rounded outward, exact leaf boxes tested before the triangles);
//   * inner nodes are walked while lanes look for a leaf (one leaf is postponed per lane), then the
//     lanes test their leaves together.  The inner phase ends once fewer than kInnerExit lanes still
//     look for a leaf and the leaf phase once fewer than kLeafExit lanes hold one: the others keep
//     their leaf or their place in the walk for the next round, so every lane visits the same nodes
//     and tests the same leaves in the same order as without the early exits;
//   * lanes whose ray has finished take a new one from the walk's queue policy (LevelQueue: one
//     wave-aggregated atomic per refill on 8 per-XCD-group cursors, once DScene::refill lanes are
//     idle; a wave-private pool for the tile kernel) instead of idling until the slowest ray of a
//     64-ray batch is done;
//   * in a queue's tail, idle lanes take pending subtrees of walking lanes of their wave (donation);
//   * the top kTopNodes inner nodes (breadth-first numbering) are read from an LDS copy;
//   * node and triangle gathers are buffer loads of exact width with 32-bit offsets.
// Planes / spheres (tiny BVHs, empty for OBJ scenes) are tested at ray fetch with the simple
// walker, area lights when the triangle walk ends, in the reference's category order.
//
// Measured alternatives (removed after A/B on MI355X): 8-wide nodes, packed
// 32-B nodes, binary16 grid indices, tail assist, trimmed grids, a last-occluder shadow probe, one
// launch for all levels, ray sorting, concurrent chunk pipelines - all result-invariant and all
// slower than this walk on the C4 frame.
#pragma once

#include "mrt_device.hpp"
#include "mrt_kernels.hpp"

namespace mrt {

constexpr int kRefDone = 0x7FFFFFFF;  // sentinel: no node (never a valid inner index)
constexpr int kWalkRefill = 32;       // idle lanes before a wave fetches new rays (DScene::refill at upload; frames set it by paths per lane)
constexpr int kWalkShards = kMaxFetchShards;  // work cursors per level (cursor c: XCD group c % 8)
// Cursors a wave tries (its own XCD group's first) before it stops fetching.  When a level's queue
// runs dry every resident wave polls the cursors it has left with an atomic each, and same-address
// atomics serialise at the memory side: a walk launch with no rays to walk took 100 us with 8
// (every wave polling every cursor), 19 us with 1 (profiles/r04_latency_probe.txt).  With each
// cursor over a contiguous eighth of the queue, 4 kept most of the load balancing between the XCD
// groups (C4 15.40 -> 15.22 ms, N = 8 shard 2.88 -> 2.85 ms; 2: 15.28 / 2.88).  With the cursors'
// interleaved chunks (below) every cursor holds a mix of cheap and costly regions, and 2 suffice:
// C4 15.06-15.10 -> 15.02-15.04 ms, N = 8 shard 2.78 -> 2.71-2.73 ms (4: 15.04 / 2.72; 1: 15.09 /
// 2.70; profiles/r04_cursor_interleave_ab.txt).
#ifndef MRT_WALK_SEGMENTS
#define MRT_WALK_SEGMENTS 2
#endif
// Cursors a workgroup tries: MRT_WALK_SEGMENTS when the grid covers every cursor's starting group
// (>= kWalkShards workgroups, the persistent grids' normal case), else all of them, so that every
// ray is walked whatever the grid size (a small shadow-grid percentage, a partition with few CUs).
__device__ __forceinline__ int walkSegments() {
    return gridDim.x >= static_cast<unsigned>(kWalkShards) ? MRT_WALK_SEGMENTS : kWalkShards;
}
constexpr int kWalkStack = kLdsStackMin;  // LDS stack entries per thread (deeper ones spill)
constexpr int kWalkTop = kTopNodesMax;
// The while-while walk's inner phase ends when fewer than this many lanes still look for a leaf
// (Aila & Laine's "while-while" waits for all of them: 1).  C4 (closest / any hit both 4): 17.51
// -> 17.29 ms, N = 8 shard 3.31 -> 3.24 ms.  Scheduling only: every lane
// walks the same nodes in the same order.
#ifndef MRT_INNER_EXIT
#define MRT_INNER_EXIT 4
#endif
#ifndef MRT_INNER_EXIT_ANY
#define MRT_INNER_EXIT_ANY MRT_INNER_EXIT
#endif
constexpr int kInnerExitClosest = MRT_INNER_EXIT;
constexpr int kInnerExitAny = MRT_INNER_EXIT_ANY;
// ... and its leaf phase once fewer than this many lanes hold a leaf (1: when all are done).  C4:
// 17.31 -> 16.66 ms, N = 8 shard 3.25 -> 3.17 ms at 12 (8: 16.68 / 3.18, 16: 16.66 / 3.20,
// 32: 16.96 / 3.30); the any-hit walk at 6 (12 / 20: +0.02 / +0.05 ms).
#ifndef MRT_LEAF_EXIT
#define MRT_LEAF_EXIT 12
#endif
#ifndef MRT_LEAF_EXIT_ANY
#define MRT_LEAF_EXIT_ANY 6
#endif
constexpr int kLeafExitClosest = MRT_LEAF_EXIT;
constexpr int kLeafExitAny = MRT_LEAF_EXIT_ANY;
// ... both scaled by the wave's lanes holding a ray (traceWhileWhileQ)
#ifndef MRT_SCALED_EXIT
#define MRT_SCALED_EXIT 1
#endif

// Buffer loads for the scene gathers: exact widths (the 8-byte child-reference load is not
// widened to 16 bytes, which costs texture-data cycles), a 32-bit VGPR offset instead of a
// 64-bit address, and the base in SGPRs.
using BufRes = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ BufRes bufferOf(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), static_cast<short>(0), 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ float4 bload4(BufRes r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ float4 bload3(BufRes r, uint32_t off) {  // xyz; w undefined
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), 0.0F);
}
__device__ __forceinline__ int2 bload2i(BufRes r, uint32_t off) {
    return __builtin_bit_cast(int2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ int4 bload4i(BufRes r, uint32_t off) {
    return __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// counting builds: one wave iteration of a walk phase and the lanes executing it (added by the
// first of them)
__device__ __forceinline__ void phaseCount(uint32_t* iters, uint32_t* lanes) {
    const uint64_t act = __ballot(true);
    if (__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(act >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(act), 0u)) == 0) {
        *iters += 1u;
        *lanes += static_cast<uint32_t>(__popcll(act));
    }
}

// a lane's walk is over (no node left, no postponed leaf)
__device__ __forceinline__ bool over2(int ref, int leaf) { return ref == kRefDone && leaf >= 0; }

// number of set bits of a wave mask below this lane
__device__ __forceinline__ int lanesBelowIn(uint64_t m) {
    return static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
}

template <class Stack>
__device__ __forceinline__ int popCulled(Stack& st, float lim, bool cull) {
    while (st.sp > 0) {
        const int2 e = st.pop();
        if (!cull || !(__int_as_float(e.y) > lim)) return e.x;
    }
    return kRefDone;
}

// ---- the conservative t-cull -------------------------------------
// The reference tests every triangle whose ancestors' boxes the ray passes (BVH.hpp:327-384);
// a box may be skipped only if no triangle inside can produce a hit the reference accepts with
// t below the current best.  Moller-Trumbore's t is NOT bounded by the triangle's box: for a
// grazing ray the determinant D = AB . (d x AC) is dominated by rounding and t_c = lambda t_plane
// with lambda = D / D_c anywhere in (0, 1) (tests/cull_cases.py).  The rounding bounds of the
// reference's own evaluation order give, for every accepted hit on a triangle T,
//     |P_c - T| <= rho,  P_c = o + t_c d,
//     rho = 4 gamma_7 |o - A|_1 |d|_1 K_T / (|d . n_T| - gamma_5 |d|_1 K_T),  K_T = |AB|_1 |AC|_1 / |AB x AC|,
// so t_c >= the entry of the ray into the box inflated by rho.  Per child the host stores a
// cone of normal lines (|n . a| >= cos psi for every triangle below) and K = max K_T
// (mrt_common.hpp, cull words); the key below is that inflated entry with
// |d . n| >= |d . a| cos psi - |d x a| sin psi and |o - A| <= |o - centre| + half diagonal.
// No bound (a cone containing a line perpendicular to d, a degenerate triangle): key 0, never culled.
__device__ __forceinline__ float cullKey(uint32_t w, float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                         float tmx, float tmy, float tmz, v3 o, v3 d, v3 inv) {
    const uint32_t qc = coneQ(w), kc = coneK(w);
    if (qc >= 127u || kc >= 127u) return 0.0F;
    const v3 a0 = coneAxis(w);
    const v3 a = a0 * (1.0F / sqrtf(dot(a0, a0)));
    const float dn = sqrtf(dot(d, d));
    const float c = fabsf(dot(d, a));
    const float sn = length(cross(d, a)) * 1.000001F + 1e-7F * dn;  // |d x a|, rounded up
    const float q = static_cast<float>(qc) * (1.0F / 126.0F);       // >= sin(psi)
    const float cq = sqrtf(fmaxf(1.0F - q * q, 0.0F)) * 0.999999F;   // <= cos(psi)
    const float smin = c * cq - sn * q;  // |d . n| >= this for every normal line in the cone
    const float K = __builtin_amdgcn_exp2f(static_cast<float>(kc) * 0.125F) * 1.0001F;
    const float dl1 = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
    // |D_c| >= |N| (|d . n| - gamma_5 |d|_1 K): 2e-6 |d| covers the float evaluation of smin
    const float den = smin - 2e-6F * dn - 0x1p-20F * K * dl1;
    if (!(den > 0.0F)) return 0.0F;
    const v3 ctr{0.5F * (mnx + mxx), 0.5F * (mny + mxy), 0.5F * (mnz + mxz)};
    const float hd = 0.5F * length(v3{mxx - mnx, mxy - mny, mxz - mnz});
    // |o - A| <= L; the absolute term covers the box's own rounding (Triangle.cpp:116-123 builds
    // it from A + AB, A + AC in float) and the centre's
    const float L = (length(o - ctr) + hd) * 1.0001F + 0x1p-20F * (fabsf(ctr.x) + fabsf(ctr.y) + fabsf(ctr.z) + hd);
    // main term: 4 gamma_5 sqrt(3) < 2^-18; + 2^-20 L for the last products' rounding
    const float rho = (0x1p-18F * K * dl1 * L / den + 0x1p-20F * L) * 1.001F;
    // entry into the box inflated by rho, per axis, each term rounded down (2^-19 relative)
    const float kx = tmx - fabsf(tmx) * 0x1p-19F - rho * fabsf(inv.x) * (1.0F + 0x1p-19F);
    const float ky = tmy - fabsf(tmy) * 0x1p-19F - rho * fabsf(inv.y) * (1.0F + 0x1p-19F);
    const float kz = tmz - fabsf(tmz) * 0x1p-19F - rho * fabsf(inv.z) * (1.0F + 0x1p-19F);
    return fmaxf(fmaxf(kx, ky), kz);
}

// The exact mode's certified leaf key (mode 3): the same bound as cullKey, evaluated from a leaf
// record precomputed on the host (mrt_scene.cpp leafCullRecord: r1.zw, r2.x = a' = a cos(psi),
// r2.y = q >= sin(psi), r2.z = Kc >= 2^-18 * 1.001 * K, r2.w = D) with cheaper, looser steps:
//   |d . n| >= |d . a| cos psi - |d x a| sin psi >= |d . a'| - q |d|_1       (|d x a| <= |d|_1)
//   den = that - (2e-6 + Kc / 4) |d|_1 <= smin - 2e-6 |d| - 2^-20 K |d|_1
//   L = te |d|_1 1.0001 + D >= |o - A| for every vertex A in the box (the ray's entry point is in it)
//   rho = L (Kc |d|_1 / den + 2^-20) 1.002 >= cullKey's rho (rcp's 1 ulp and the 2^-19 of the
//   inflation included), key = the entry of the box inflated by rho, per axis, rounded down.
// Every float step rounds at most a few ulps against margins of >= 2^-19 relative.  key <= te.
__device__ __forceinline__ float leafKey(float4 r1, float4 r2, float te, float ex, float ey, float ez, v3 d, v3 inv) {
    const float dl1 = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
    const float c = fabsf(fmaf(d.z, r2.x, fmaf(d.y, r1.w, d.x * r1.z)));
    const float den = c - dl1 * (r2.y + fmaf(0.25F, r2.z, 2e-6F));
    if (!(den > 0.0F)) return 0.0F;
    const float L = fmaf(te, dl1 * 1.0001F, r2.w);
    const float rho = L * fmaf(r2.z * dl1, __builtin_amdgcn_rcpf(den), 0x1p-20F) * 1.002F;
    const float kx = fmaf(-rho, fabsf(inv.x), fmaf(-0x1p-19F, fabsf(ex), ex));
    const float ky = fmaf(-rho, fabsf(inv.y), fmaf(-0x1p-19F, fabsf(ey), ey));
    const float kz = fmaf(-rho, fabsf(inv.z), fmaf(-0x1p-19F, fabsf(ez), ez));
    return fmaxf(fmaxf(kx, ky), kz);
}

// Culling against the keys, near-first order (by box entry) and the push of the far child.
template <class Stack>
__device__ __forceinline__ int chooseChildren(bool hl, bool hr, float tl, float tr, float kl, float kr, int refL,
                                              int refR, float lim, bool cull, Stack& st, bool rightFirst) {
    if (cull) {
        hl = hl && !(kl > lim);
        hr = hr && !(kr > lim);
    }
    if (hl && hr) {
        int nearRef = refL, farRef = refR;
        float farK = kr;
        if (cull && rightFirst) {
            nearRef = refR;
            farRef = refL;
            farK = kl;
        }
        st.push(farRef, farK);
        return nearRef;
    }
    if (hl) return refL;
    if (hr) return refR;
    return popCulled(st, lim, cull);
}

// Cull modes (DScene::cull, mrt_set_tuning key 2):
//   0  no culling: exactly the reference's visit set;
//   1  fast: skip a box whose entry exceeds best * (1 + 2^-10).  Exact unless a triangle inside
//      is hit at a grazing angle (|d . n| below ~1e-3) whose rounding moves Moller-Trumbore's t
//      below the best hit (tests/cull_cases.py builds one); NOT exact for every input;
//   2  certified: the keys of cullKey (a rigorous lower bound on every acceptable t below the
//      box) on every node of the reference tree, exact for every input; slow (the bound needs
//      each child's normal cone, and the cones of closed objects hold every direction);
//   3  exact (default): the inner nodes of the quantized 4-wide tree are never culled (mode 0's
//      visit set), and a leaf whose exact box passes is skipped only when its certified key
//      (cullKey over the leaf's own <= 4 triangles, whose cone is narrow) exceeds the best:
//      exact for every input, and the triangle tests behind the best hit are mostly avoided.
constexpr int kCullNone = 0, kCullFast = 1, kCullCertified = 2, kCullExact = 3;
constexpr float kCullMargin = 0x1p-10f;  // cull mode 1

// the limit a key is compared with: a child / stack entry is skipped iff key > limit
template <int kCull>
__device__ __forceinline__ float cullLimit(float best) {
    return kCull == kCullFast ? best + best * kCullMargin : best;
}
// modes that cull inner nodes and stack entries (mode 3 culls leaves only)
template <int kCull>
constexpr int innerCullMode() {
    return (kCull == kCullFast || kCull == kCullCertified) ? kCull : kCullNone;
}

// One BVH2 inner-node visit: returns the next node (near child, or a popped entry).
// Reference-tree nodes (GNode, exact boxes, from global memory).
// finite: wave-uniform, every active lane's 1/d is finite (slabFinite applies; otherwise the
// exact slab, and the certified mode does not cull)
template <int kCull, class Stack>
__device__ __forceinline__ int innerStep(BufRes nodes, int ref, v3 o, v3 d, v3 inv, float lim, Stack& st,
                                         TravCount* cnt, bool count, bool finite, int order) {
    constexpr bool cull = kCull != kCullNone;
    const uint32_t off = static_cast<uint32_t>(ref) * static_cast<uint32_t>(sizeof(GNode));
    const float4 n0 = bload4(nodes, off);
    const float4 n1 = bload4(nodes, off + 16u);
    const float4 n2 = bload4(nodes, off + 32u);
    int4 n3;
    if (kCull == kCullCertified) {
        n3 = bload4i(nodes, off + 48u);  // child refs and cull words
    } else {
        const int2 r = bload2i(nodes, off + 48u);  // child refs
        n3 = make_int4(r.x, r.y, 0, 0);
    }
    if (count) cnt->nodes += 2;
    float tl, tr, kl = 0.0F, kr = 0.0F;
    bool hl, hr;
    if (kCull != kCullCertified) {
        if (finite) {
            hl = slabFinite(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, o, inv, &tl);
            hr = slabFinite(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, o, inv, &tr);
        } else {
            hl = slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, o, inv, &tl);
            hr = slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, o, inv, &tr);
        }
        kl = tl;
        kr = tr;
    } else if (finite) {
        float lx, ly, lz, rx, ry, rz;
        hl = slabFiniteAxes(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, o, inv, &tl, &lx, &ly, &lz);
        hr = slabFiniteAxes(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, o, inv, &tr, &rx, &ry, &rz);
        // keys are needed for a child that may be culled now (entry beyond the best hit; a key
        // never exceeds the entry) and for the far child, which goes on the stack
        const bool rFar = !(tr < tl);
        if (cull && hl && (tl > lim || (hr && !rFar)))
            kl = cullKey(static_cast<uint32_t>(n3.z), n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, lx, ly, lz, o, d, inv);
        if (cull && hr && (tr > lim || (hl && rFar)))
            kr = cullKey(static_cast<uint32_t>(n3.w), n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, rx, ry, rz, o, d, inv);
    } else {
        hl = slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, o, inv, &tl);
        hr = slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, o, inv, &tr);
    }
    // both children hit (culling modes): the nearer entry first (order 0), or the farther (1).  Shadow
    // rays walk far first by default: an occluder between a surface point and the light is found
    // sooner from the light's side on the Conference frame (-2 % frame time);
    // the order changes which occluder is found first, never whether one is
    const bool rightFirst = order == 0 ? tr < tl : !(tr < tl);
    return chooseChildren(hl, hr, tl, tr, kl, kr, n3.x, n3.y, lim, cull, st, rightFirst);
}

// The quantized walk tree's planes: t = fma(q, qa, qb) with qa = step / d, qb = (origin - o) / d
// per axis (rounded as the Quantizer's bound in mrt_scene.cpp assumes); the slab logic of slabFinite.
// This form (the packet walk's) takes the bounds as floats, min xyz then max xyz.
__device__ __forceinline__ bool qslab(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, v3 qa, v3 qb,
                                      float* tEntry) {
    const float t1x = fmaf(mnx, qa.x, qb.x), t2x = fmaf(mxx, qa.x, qb.x);
    const float t1y = fmaf(mny, qa.y, qb.y), t2y = fmaf(mxy, qa.y, qb.y);
    const float t1z = fmaf(mnz, qa.z, qb.z), t2z = fmaf(mxz, qa.z, qb.z);
    const float e = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fmaxf(fminf(t1z, t2z), 0.0F));
    const float tMax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
    *tEntry = e;
    return tMax >= e;
}
// The per-lane walk's form on the node's words.  A child's axis is one word, min | max << 16
// (QNode4).  For qa > 0 the min plane is the nearer one: fma is monotone in q (correctly rounded),
// so min(t(min), t(max)) = t(min); for qa < 0 the max plane.  The word is rotated by 16 bits when
// the axis's 1/d is negative (nearFarShift, one v_alignbit), after which its low half is the near
// plane and its high half the far one: the same entry and exit without the three min / max pairs
// (19 VALU per child instead of 22).  quantOK rays have finite, nonzero qa and qb: no NaN.
__device__ __forceinline__ uint32_t nearFarShift(float qa) { return (__float_as_uint(qa) >> 27) & 16u; }
__device__ __forceinline__ bool qslabNF(uint32_t wx, uint32_t wy, uint32_t wz, uint32_t sx, uint32_t sy, uint32_t sz,
                                        v3 qa, v3 qb, float* tEntry) {
    const uint32_t rx = __builtin_amdgcn_alignbit(wx, wx, sx);
    const uint32_t ry = __builtin_amdgcn_alignbit(wy, wy, sy);
    const uint32_t rz = __builtin_amdgcn_alignbit(wz, wz, sz);
    const float nx = fmaf(static_cast<float>(rx & 0xFFFFu), qa.x, qb.x), fx = fmaf(static_cast<float>(rx >> 16), qa.x, qb.x);
    const float ny = fmaf(static_cast<float>(ry & 0xFFFFu), qa.y, qb.y), fy = fmaf(static_cast<float>(ry >> 16), qa.y, qb.y);
    const float nz = fmaf(static_cast<float>(rz & 0xFFFFu), qa.z, qb.z), fz = fmaf(static_cast<float>(rz >> 16), qa.z, qb.z);
    const float e = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.0F));
    const float tMax = fminf(fminf(fx, fy), fz);
    *tEntry = e;
    return tMax >= e;
}

// compare-exchange of two (sort key, reference) pairs: ascending keys
__device__ __forceinline__ void cex(float& ka, int& ra, float& kb, int& rb) {
    const bool sw = kb < ka;
    const float k = sw ? kb : ka;
    const int r = sw ? rb : ra;
    kb = sw ? ka : kb;
    rb = sw ? ra : rb;
    ka = k;
    ra = r;
}

// ascending sort of kWalkWidth (key, reference) pairs: Batcher's odd-even merge networks
template <int W>
__device__ __forceinline__ void sortChildren(float* k, int* r) {
    if (W == 4) {
        cex(k[0], r[0], k[1], r[1]);
        cex(k[2], r[2], k[3], r[3]);
        cex(k[0], r[0], k[2], r[2]);
        cex(k[1], r[1], k[3], r[3]);
        cex(k[1], r[1], k[2], r[2]);
    } else {
        constexpr int net[19][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3}, {4, 6}, {5, 7}, {1, 2}, {5, 6},
                                    {0, 4}, {1, 5}, {2, 6}, {3, 7}, {2, 4}, {3, 5}, {1, 2}, {3, 4}, {5, 6}};
#pragma unroll
        for (int c = 0; c < 19; ++c) cex(k[net[c][0]], r[net[c][0]], k[net[c][1]], r[net[c][1]]);
    }
}

// One walk-tree visit (QNode4: kWalkWidth 16-byte loads, or LDS for the top nodes).  Every child
// box holds the reference leaf boxes below it with the Quantizer's margin (mrt_scene.cpp), so for
// the rays admitted to this tree a child passes whenever a leaf below passes the reference test,
// and its entry is at most that leaf's: the visit set is a superset of the reference's, and the
// leaves are tested exactly before their triangles (traceWhileWhile).  The hit children are
// visited in order of entry (kOrder 0: nearest first; 1: farthest first, a compile-time choice
// made per wave from the uniform DScene::anyOrder): the first now, the others pushed.
template <int kCull, int kOrder, class Stack>
__device__ __forceinline__ int innerStepQ(BufRes qnodes, const QNode4* ldsTop, int top, int ref, v3 qa, v3 qb,
                                          float lim, Stack& st, TravCount* cnt, bool count) {
    constexpr int W = kWalkWidth;
    constexpr bool cull = kCull != kCullNone;
    int4 raw[W];
    if (ref < top) {
        const int4* np = reinterpret_cast<const int4*>(ldsTop + ref);
#pragma unroll
        for (int j = 0; j < W; ++j) raw[j] = np[j];
    } else {
        const uint32_t off = static_cast<uint32_t>(ref) * static_cast<uint32_t>(sizeof(QNode4));
#pragma unroll
        for (int j = 0; j < W; ++j) raw[j] = bload4i(qnodes, off + 16u * static_cast<uint32_t>(j));
    }
    const auto word = [&](int i) -> uint32_t {  // word i of the node (i a compile-time constant after unrolling)
        const int4 v = raw[i >> 2];
        const int c = i & 3;
        return static_cast<uint32_t>(c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w);
    };
    constexpr float kInf = __builtin_inff();
    const uint32_t sx = nearFarShift(qa.x), sy = nearFarShift(qa.y), sz = nearFarShift(qa.z);
    constexpr float sg = kOrder == 0 ? 1.0F : -1.0F;  // sort keys: the entry (nearest first) or its negation
    float key[W];
    int rf[W];
    int n = 0;
#pragma unroll
    for (int c = 0; c < W; ++c) {
        const uint32_t w0 = word(3 * c), w1 = word(3 * c + 1), w2 = word(3 * c + 2);
        rf[c] = static_cast<int>(word(3 * W + c));
        if (count) cnt->nodes += rf[c] != kEmptyChild ? 1u : 0u;
        float t;
        // (an unused slot holds an inverted box, which this test misses: near > far on every axis,
        // since |qb| <= 4 * 65535 |qa| for quantOK rays keeps fma(65535, qa, qb) != qb)
        bool h = qslabNF(w0, w1, w2, sx, sy, sz, qa, qb, &t);
        if (cull) h = h && !(t > lim);
        n += h ? 1 : 0;
        key[c] = h ? sg * t : kInf;  // misses last
    }
    if (n == 0) return popCulled(st, lim, cull);
    sortChildren<W>(key, rf);
    // push the others farthest-in-order first (a keyed stack's key is the entry, for popCulled)
#pragma unroll
    for (int k = W - 1; k >= 1; --k)
        if (k < n) st.push(rf[k], sg * key[k]);
    return rf[0];
}

// A ray may walk the quantized tree when the Quantizer's bound (mrt_scene.cpp) holds for it: every 1/d
// component in [2^-40, 2^90], qa = step / d normal (>= 2^-100: an unused slot's inverted box then
// always misses, innerStepQ) and the origin within 4 grid extents of the grid origin per axis.
__device__ __forceinline__ bool quantOK(const DScene& s, v3 o, v3 inv) {
    if (s.qEnabled == 0) return false;
    const float ov[3] = {o.x, o.y, o.z}, iv[3] = {inv.x, inv.y, inv.z};
    bool ok = true;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float ai = fabsf(iv[a]);
        ok = ok && ai >= 0x1p-40F && ai <= 0x1p90F && ai * s.qgrid.step[a] >= 0x1p-100F &&
             fabsf(ov[a] - s.qgrid.origin[a]) <= 4.0F * 65535.0F * s.qgrid.step[a];
    }
    return ok;
}

// Copies the walk tree's top into LDS (all threads; ends with a barrier).
template <int kThreads>
__device__ __forceinline__ void stageTop(const DScene& s, QNode4* ldsTop) {
    const int n = min(kWalkTop, s.triTop) * static_cast<int>(sizeof(QNode4) / sizeof(float4));
    const float4* src = reinterpret_cast<const float4*>(s.triQNodes);
    float4* dst = reinterpret_cast<float4*>(ldsTop);
    for (int i = static_cast<int>(threadIdx.x); i < n; i += kThreads) dst[i] = src[i];
    __syncthreads();
}

// The work cursors' layout (round 4).  Cursor s serves the chunks s, s + 8, s + 16, ... of 2^shift
// queue entries, not a contiguous eighth of the queue: adjacent entries are spatially coherent, so
// a contiguous eighth is one region of the image, and the regions' costs differ - a cursor over
// cheap pixels ran dry early, and the waves that had drained their cursors ended while the others
// still walked (at the N = 8 shard a level's waves ended between 38 % and 74 % of it).  Chunks of
// 4,096 rays keep a wave's rays coherent; at least 8 chunks per cursor keep small queues spread.
#ifndef MRT_SEG_INTERLEAVE
#define MRT_SEG_INTERLEAVE 1
#endif
// The cursors hand out the queue from its end (round 5): a level's queue is written in index order
// by the shading before it, so its last entries are the most recently written and, at N = 1 (each
// level's ray records ~400 MB, more than the 256 MB Infinity Cache), the ones still cached.  C4
// 14.655 -> 14.575 ms, N = 8 shard unchanged (2.63 / 2.64 ms; its queues fit the cache), images
// identical (profiles/r05_queue_order_ab.txt).
// The leaf loop's triangles software-pipelined (round 5): triangle k + 1's three loads go out
// before triangle k's test, so a lane's tests wait on one round trip per leaf instead of one per
// triangle.  It needs 9 more VGPRs across the test, which the walks' 6 waves per SIMD (80 VGPRs,
// mrt_kernels.hip MRT_WALK_WAVES) hold: C4 14.53 -> 14.05 ms, N = 8 shard 2.61 -> 2.53 ms, the flat
// stand-in 39.4 -> 37.7 ms, images identical (profiles/r05_tri_prefetch_ab.txt; at 7 waves it spilled
// 36 B and lost).
#ifndef MRT_TRI_PREFETCH
#define MRT_TRI_PREFETCH 1
#endif
#ifndef MRT_TRI_PREFETCH_ANY
#define MRT_TRI_PREFETCH_ANY MRT_TRI_PREFETCH  // the any-hit (shadow) walk's
#endif
#ifndef MRT_SEG_REVERSE
#define MRT_SEG_REVERSE 1
#endif
// The leaf phase's triangles spread over the wave (round 6, MRT_TRI_SPREAD = 1, default): the leaf
// phase wave-uniform, each lane testing its leaf's first triangle itself (loaded with the leaf box)
// and the leaves' further triangles spread over all 64 lanes, one (owner, triangle) pair per lane and
// round, results merged by each owner in its own triangle order - the per-lane loop's results bit
// for bit.  Spill-free at 80 VGPRs (no prefetch; qa, qb recomputed per inner phase).  Flat stand-in
// 37.7 -> 36.5 ms, its N = 8 shard 7.36 -> 7.02 ms, the Conference stand-in within +-0.5 % (13.91 /
// 13.97 ms, N = 8 2.52 / 2.51 ms); closest-hit triangle-loop lane use 0.35 -> 0.54
// (profiles/r06_tri_spread_ab.txt).  0: the per-lane loop with the prefetch above.  (Round 5's form,
// which spilled 44-68 B at 72 VGPRs, lost everywhere.)
#ifndef MRT_TRI_SPREAD
#define MRT_TRI_SPREAD 1
#endif
#ifndef MRT_TRI_SPREAD_ANY
#define MRT_TRI_SPREAD_ANY MRT_TRI_SPREAD  // the any-hit (shadow) walk's
#endif
#ifndef MRT_SEG_CHUNK_LOG
#define MRT_SEG_CHUNK_LOG 12
#endif
constexpr int kSegChunkLog = MRT_SEG_CHUNK_LOG;  // rays per chunk: 2^12
// log2 of the chunk size for n entries: maxLog, or smaller so that every cursor has >= 8 chunks
__device__ __forceinline__ int segChunkShift(int n, int maxLog) {
    const int per = max(n >> 6, 1);  // n / (8 cursors x 8 chunks)
    return min(maxLog, 31 - __clz(per));
}
// the queue entry of cursor seg's j-th claim
__device__ __forceinline__ int interleavedIndex(int j, int seg, int shift) {
    return ((((j >> shift) * kWalkShards) + seg) << shift) + (j & ((1 << shift) - 1));
}

// The rays a walk takes: a queue policy.
//   o(i), d(i)      ray i's origin / direction records;
//   hit(i, h)       the closest hit (t, u, v, primitive code); occ(i, f): the occluded flag;
//   take(pending)   called by every lane of the wave (wave-uniform control flow) with the mask of
//                   lanes wanting a ray: this lane's ray index, or -1 (none left for it);
//   drained()       wave-uniform: the queue has no ray left for this wave.
// LevelQueue: a level's queue arrays, rays [0, count), fetched through kWalkShards cursors
// (kFetchStride ints apart), one per XCD group of workgroups (blockIdx % 8), each over its
// interleaved chunks of the queue (above); a drained cursor is left for the next (speed only: any
// placement gives the same results).
// Round 6: with queue segments (kQueueSegs == kWalkShards, mrt_kernels.hpp) cursor s serves segment
// s - the rays k_shade's workgroups b % 8 == s allocated, a mix of the image like the interleaved
// chunks - from its most recently written end; with one segment the interleaved chunks above.
static_assert(kQueueSegs == 1 || kWalkShards % kQueueSegs == 0, "queue segments: whole cursors each");
struct LevelQueue {
    const float4* __restrict__ rO;
    const float4* __restrict__ rD;
    float4* out;
    SegMap map;
    int count;
    int* fetch;
    int seg = static_cast<int>(blockIdx.x % kWalkShards);  // wave-uniform cursor state
    int segsLeft = walkSegments();
    int shift;  // the cursors' chunks: 2^shift rays
    __device__ __forceinline__ LevelQueue(const float4* o_, const float4* d_, float4* out_, const SegMap& map_, int* fetch_)
        : rO(o_), rD(d_), out(out_), map(map_), count(map_.total()), fetch(fetch_),
          shift(segChunkShift(map_.total(), kSegChunkLog)) {}
    // segment g's ray count (g wave-uniform)
    __device__ __forceinline__ int segCount(int g) const {
        int c = 0;
#pragma unroll
        for (int k = 0; k < kQueueSegs; ++k)
            if (k == g) c = map.pre[k + 1] - map.pre[k];
        return c;
    }
    __device__ __forceinline__ float4 o(int i) const { return rO[i]; }
    __device__ __forceinline__ float4 d(int i) const { return rD[i]; }
    __device__ __forceinline__ void hit(int i, float4 h) const { out[i] = h; }
    __device__ __forceinline__ void occ(int i, float f) const { out[i].w = f; }
    __device__ __forceinline__ bool drained() const { return segsLeft == 0; }
    __device__ __forceinline__ int take(uint64_t pending) {
        const int lane = static_cast<int>(threadIdx.x & 63u);
        int got = -1;
        while (pending != 0 && segsLeft > 0) {
            const int n = __popcll(pending);
            const int leader = __ffsll(static_cast<unsigned long long>(pending)) - 1;
            const int segStart = static_cast<int>((static_cast<long long>(count) * seg) / kWalkShards);
            const int segEnd = static_cast<int>((static_cast<long long>(count) * (seg + 1)) / kWalkShards);
            int base = 0;
            if (lane == leader) base = atomicAdd(fetch + seg * kFetchStride, n);
            base = __shfl(base, leader, 64);
            const bool mine = ((pending >> lane) & 1ull) != 0;
            if (kQueueSegs > 1) {
                (void)segStart;
                (void)segEnd;
                // cursor seg: segment seg % kQueueSegs, its part seg / kQueueSegs of kWalkShards / kQueueSegs
                constexpr int kParts = kWalkShards / kQueueSegs;
                const int g = seg % kQueueSegs, part = seg / kQueueSegs;
                const int cnt = segCount(g);
                const int lo = static_cast<int>((static_cast<long long>(cnt) * part) / kParts);
                const int hi = static_cast<int>((static_cast<long long>(cnt) * (part + 1)) / kParts);
                const int idx = base + lanesBelowIn(pending);
                if (mine && idx < hi - lo) got = g * map.segCap + (hi - 1 - idx);  // most recently written first
            } else if (mine) {
#if MRT_SEG_INTERLEAVE
                (void)segStart;
                (void)segEnd;
                const int idx = interleavedIndex(base + lanesBelowIn(pending), seg, shift);
#if MRT_SEG_REVERSE
                if (idx < count) got = count - 1 - idx;
#else
                if (idx < count) got = idx;
#endif
#else
                const int idx = segStart + base + lanesBelowIn(pending);
                if (idx < segEnd) got = idx;
#endif
            }
            pending = __ballot(mine && got < 0);
            if (pending != 0) {
                seg = (seg + 1) % kWalkShards;
                --segsLeft;
            }
        }
        return got;
    }
};

// kAny = false: closest hit -> q.hit(i, (t, u, v, primitive code));
// kAny = true:  shadow any-hit -> q.occ(i, occluded flag).
template <bool kAny, bool kCount, int kCull, class Stack, class Queue>
__device__ __forceinline__ void traceWhileWhileQ(const DScene& s, Queue& q, Stack& st, TravCount* cnt,
                                                 const QNode4* ldsTop, int* tailBest) {
    // MRT_TRI_SPREAD for this walk: 0 the per-lane triangle loop, 1 the spread tests
    constexpr int kSpread = kAny ? MRT_TRI_SPREAD_ANY : MRT_TRI_SPREAD;
    __shared__ uint8_t spreadOwners[kSpread != 0 ? 192 * 4 : 1];  // per wave: the owner lane of each spread test
    constexpr int kHelper = -2;  // rayIdx of a lane walking a subtree given by another lane
    const bool donate = s.tailDonate != 0;
    const int top = min(kWalkTop, s.triTop);
    const BufRes nodeBuf = bufferOf(s.triNodes);
    const BufRes qBuf = bufferOf(s.triQNodes);
    const BufRes triBuf = bufferOf(s.triGeom);
    const BufRes leafBuf = bufferOf(s.leafBoxes);
    constexpr int kInner = innerCullMode<kCull>();  // the cull mode of inner nodes and pops
    constexpr bool cull = kInner != kCullNone;
    const int lane = static_cast<int>(threadIdx.x & 63u);
    int rayIdx = -1;
    bool exhausted = false;
    v3 o{0, 0, 0}, d{0, 0, 0}, inv{0, 0, 0};
    v3 qa{0, 0, 0}, qb{0, 0, 0};  // quantized walk tree: t = fma(q, qa, qb) (innerStepQ)
    bool refTree = true;          // this lane walks the reference tree (GNode) instead
    uint32_t src = 0;
    // closest hit so far: t and primitive code only; u, v are recomputed for the winner at
    // the end (same inputs -> same bits), which keeps two registers out of the walk
    float bt = kRayLengthMax;
    uint32_t bcode = kNoPrim;
    int ref = kRefDone;
    int leaf = 0;  // < 0: a postponed leaf
    // tail donation (DScene::tailDonate): a helper lane walks a subtree of its owner's ray and
    // hands its best hit (closest) or occlusion (any) back; the owner finishes when all its
    // helpers have.  Exact: the owner and its helpers visit the owner's subtrees between them,
    // each culling against a best no better than the final one, and betterThan is a total order.
    // In tail mode an owner and its helpers share, through the owner's LDS word in tailBest, the
    // best t any of them has accepted (closest hit: the cull limit of all of them; it is the t of an
    // accepted candidate, so never below the final best) or the occlusion (any-hit: 0, they stop).
    int owner = -1;     // helper: the lane owning the ray
    int pend = 0;       // owner: helpers still walking
    bool occ = false;   // any-hit: an occluder found (by this lane, or merged from a helper)
    bool tailMode = false;  // wave-uniform: this wave has donated (its queue is exhausted)
    float shT = __builtin_inff();  // tail mode: the best t shared by the ray's lanes
    int* const waveBest = tailBest + (threadIdx.x & ~63u);
    while (true) {
        if (tailMode && rayIdx != -1) {
            const int ol = rayIdx >= 0 ? lane : owner;
            const int mine = kAny ? (occ ? 0 : 0x7FFFFFFF) : __float_as_int(bt);
            const int v = min(atomicMin(waveBest + ol, mine), mine);
            if (kAny) {
                if (v == 0 && !occ) {  // another lane of this ray found an occluder: stop
                    occ = rayIdx >= 0;
                    st.sp = 0;
                    ref = kRefDone;
                    leaf = 0;
                }
            } else {
                shT = __int_as_float(v);
            }
        }
        const bool over = ref == kRefDone && leaf >= 0;
        if (donate) {  // helpers whose subtree is done merge into their owner (wave-uniform loop)
            uint64_t hm = __ballot(rayIdx == kHelper && over);
            while (hm != 0) {
                const int h = __ffsll(static_cast<unsigned long long>(hm)) - 1;
                hm &= hm - 1;
                const int ol = __builtin_amdgcn_readlane(owner, h);
                const float ht = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bt), h));
                const uint32_t hc = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(bcode), h));
                const int ho = __builtin_amdgcn_readlane(occ ? 1 : 0, h);
                if (lane == ol) {
                    if (kAny) {
                        occ = occ || ho != 0;
                    } else if (betterThan(ht, hc, bt, bcode)) {
                        bt = ht;
                        bcode = hc;
                    }
                    --pend;
                }
            }
            if (rayIdx == kHelper && over) {
                rayIdx = -1;
                occ = false;
            }
        }
        // ---- lanes whose triangle walk is over: lights (closest only), write the result ----
        // Closest hit: the lights' test and the winner's u, v cost the wave dependent loads, so
        // finished lanes wait (idle, like lanes waiting for a refill) and are completed together
        // once they and the idle lanes would trigger a refill, no lane is still walking, or the
        // queue has run dry.
        const bool doneLane = rayIdx >= 0 && over && pend == 0;
        bool runDone = true;
        if (!kAny) {
            const int nReady = __popcll(__ballot(doneLane || (rayIdx == -1 && !exhausted)));
            runDone = nReady >= s.refill || __ballot(rayIdx >= 0 && !doneLane) == 0 || __ballot(exhausted) != 0;
        }
        if (doneLane && runDone) {
            if (kCount) cnt->rayMax = max(cnt->rayMax, cnt->nodes - cnt->rayStart);
            if (kAny) {
                q.occ(rayIdx, occ ? 1.0F : 0.0F);
                if (kCount) cnt->occluded += occ ? 1u : 0u;
                occ = false;
            } else {
                for (int j = 0; j < s.nLights; ++j) {  // Shader.cpp:166-171
                    const float4* l = s.lights + 4 * j;
                    const float4 a4 = l[0];
                    if (__float_as_int(a4.w) != 1) continue;
                    float t, u, v;
                    if (!triTest(a4, l[1], l[2], o, d, &t, &u, &v)) continue;
                    if (t < kEpsilon) continue;
                    const uint32_t code = encodePrim(kLight, static_cast<uint32_t>(j));
                    if (betterThan(t, code, bt, bcode)) {
                        bt = t;
                        bcode = code;
                    }
                }
                float u = 0.0F, v = 0.0F, t;  // planes / spheres: 0, 0
                const uint32_t kind = primKind(bcode);
                if (kind == kTriangle || kind == kLight) {
                    const float4* g = kind == kTriangle ? s.triGeom + 3 * primIndex(bcode) : s.lights + 4 * primIndex(bcode);
                    (void)triTest(g[0], g[1], g[2], o, d, &t, &u, &v);
                }
                q.hit(rayIdx, make_float4(bt, u, v, bitsf(bcode)));
            }
            rayIdx = -1;
        }
        // ---- refill lanes without a ray (one atomic per wave and cursor) ----
        bool need = rayIdx == -1 && !exhausted;
        uint64_t needMask = __ballot(need);
        // refill only once enough lanes are idle (fewer, larger fetches), or when none is busy
        if (__popcll(needMask) < s.refill && __ballot(rayIdx >= 0) != 0) {
            need = false;
            needMask = 0;
        }
        if (needMask != 0) {
            const int got = q.take(needMask);
            if (need) {
                rayIdx = got;
                if (kCount) {
                    cnt->rayStart = cnt->nodes;
                    if (got >= 0) ++cnt->rays;
                }
                if (rayIdx < 0) {
                    exhausted = true;
                } else {
                    const float4 o4 = q.o(rayIdx);
                    const float4 d4 = q.d(rayIdx);
                    o = xyz(o4);
                    d = xyz(d4);
                    inv = v3{1.0F / d.x, 1.0F / d.y, 1.0F / d.z};
                    Best b;
                    if (kAny) {
                        src = fbits(o4.w);
                        b = Best{d4.w, 0.0F, 0.0F, kNoPrim};
                        bool occ = traverse<kPlane, true>(s, s.planeNodes, s.planeRoot, o, d, inv, src, &b, st, cnt);
                        occ = occ || traverse<kSphere, true>(s, s.sphereNodes, s.sphereRoot, o, d, inv, src, &b, st, cnt);
                        if (occ) {
                            q.occ(rayIdx, 1.0F);
                            rayIdx = -1;
                            if (kCount) ++cnt->occluded;
                        }
                    } else {
                        src = fbits(d4.w);
                        b = Best{kRayLengthMax, 0.0F, 0.0F, kNoPrim};
                        traverse<kPlane, false>(s, s.planeNodes, s.planeRoot, o, d, inv, src, &b, st, cnt);
                        traverse<kSphere, false>(s, s.sphereNodes, s.sphereRoot, o, d, inv, src, &b, st, cnt);
                    }
                    bt = b.t;
                    bcode = b.code;
                    if (rayIdx >= 0) {
                        float te;
                        const GRoot& r = s.triRoot;  // both trees have the same root box
                        // rays outside the quantized tree's error bound (a non-finite or extreme
                        // 1/d, a far origin) and the certified cull (its bounds are the reference
                        // nodes') walk the reference tree (DScene::triRootRef)
                        refTree = kCull == kCullCertified || !quantOK(s, o, inv);
                        if (!refTree) {
                            qa = v3{s.qgrid.step[0] * inv.x, s.qgrid.step[1] * inv.y, s.qgrid.step[2] * inv.z};
                            qb = v3{(s.qgrid.origin[0] - o.x) * inv.x, (s.qgrid.origin[1] - o.y) * inv.y,
                                    (s.qgrid.origin[2] - o.z) * inv.z};
                        }
                        if (r.count > 0 &&
                            slab(r.bmin[0], r.bmin[1], r.bmin[2], r.bmax[0], r.bmax[1], r.bmax[2], o, inv, &te)) {
                            ref = refTree ? s.triRootRef.ref : r.ref;
                            if (ref < 0) {  // the root is a leaf
                                leaf = ref;
                                ref = kRefDone;
                            }
                        }
                    }
                }
            }
        }
        // ---- a level's tail: idle lanes take the next pending subtree of a walking lane ----
        if (donate) {
            uint64_t idle = __ballot(rayIdx == -1 && (exhausted || q.drained()));
            if (idle != 0 && !tailMode) {  // the owners' shared words
                tailMode = true;
                if (rayIdx >= 0) waveBest[lane] = kAny ? 0x7FFFFFFF : __float_as_int(bt);
            }
            uint64_t donors = 0;
            for (int round = 0; idle != 0 && round < 64; ++round) {
                if (donors == 0) {
                    donors = __ballot(rayIdx != -1 && st.sp > 0);
                    if (donors == 0) break;
                }
                const int dl = __ffsll(static_cast<unsigned long long>(donors)) - 1;
                donors &= donors - 1;  // one subtree per donor and sweep
                int2 e = make_int2(kRefDone, 0);
                if (lane == dl) e.x = popCulled(st, cullLimit<kInner>(fminf(bt, shT)), cull);  // its next subtree
                const int er = __builtin_amdgcn_readlane(e.x, dl);
                if (er == kRefDone) continue;
                const int h = __ffsll(static_cast<unsigned long long>(idle)) - 1;
                idle &= idle - 1;
                const int dOwner = __builtin_amdgcn_readlane(rayIdx >= 0 ? lane : owner, dl);
                const float ox = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(o.x), dl));
                const float oy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(o.y), dl));
                const float oz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(o.z), dl));
                const float dx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d.x), dl));
                const float dy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d.y), dl));
                const float dz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d.z), dl));
                const int dsrc = __builtin_amdgcn_readlane(static_cast<int>(src), dl);
                const int dref = __builtin_amdgcn_readlane(refTree ? 1 : 0, dl);
                const float dbt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bt), dl));
                const int dbc = __builtin_amdgcn_readlane(static_cast<int>(bcode), dl);
                if (lane == h) {
                    rayIdx = kHelper;
                    owner = dOwner;
                    o = v3{ox, oy, oz};
                    d = v3{dx, dy, dz};
                    inv = v3{1.0F / d.x, 1.0F / d.y, 1.0F / d.z};
                    refTree = dref != 0;
                    if (!refTree) {  // the donor's values (same inputs, same roundings)
                        qa = v3{s.qgrid.step[0] * inv.x, s.qgrid.step[1] * inv.y, s.qgrid.step[2] * inv.z};
                        qb = v3{(s.qgrid.origin[0] - o.x) * inv.x, (s.qgrid.origin[1] - o.y) * inv.y,
                                (s.qgrid.origin[2] - o.z) * inv.z};
                    }
                    src = static_cast<uint32_t>(dsrc);
                    bt = dbt;
                    bcode = static_cast<uint32_t>(dbc);
                    shT = dbt;
                    occ = false;
                    st.sp = 0;
                    if (er < 0) {  // a leaf
                        leaf = er;
                        ref = kRefDone;
                    } else {
                        leaf = 0;
                        ref = er;
                    }
                }
                if (lane == dOwner) ++pend;
            }
        }
        const uint64_t activeMask = __ballot(rayIdx != -1);
        if (activeMask == 0) {
            if (__ballot(!exhausted) == 0) break;
            continue;
        }
        // The phases' early exits scale with the lanes that hold a ray: in a queue's tail, with a few
        // rays left in the wave, a fixed threshold would end each phase after one step and pay the
        // outer loop's refill / donation bookkeeping per node visit (scheduling only: every lane visits
        // the same nodes and tests the same leaves in the same order).
        constexpr int kExit = kAny ? kInnerExitAny : kInnerExitClosest;
        constexpr int kLeafExit = kAny ? kLeafExitAny : kLeafExitClosest;
#if MRT_SCALED_EXIT
        const int nActive = __popcll(activeMask);
        const int innerExit = max(1, (kExit * nActive + 63) >> 6);
        const int leafExit = max(1, (kLeafExit * nActive + 63) >> 6);
#else
        const int innerExit = kExit, leafExit = kLeafExit;
#endif
        // ---- inner nodes until every active lane holds a postponed leaf ----
        // (counting builds: the wave's lanes without a ray and with a finished one, per inner iteration)
        const uint32_t idleLanes = kCount ? static_cast<uint32_t>(__popcll(__ballot(rayIdx == -1))) : 0u;
        const uint32_t doneLanes = kCount ? static_cast<uint32_t>(__popcll(__ballot(rayIdx != -1 && over2(ref, leaf)))) : 0u;
        // the spread leaf phase: qa, qb recomputed per inner phase from o and 1/d (the same operations,
        // the same bits), so that they hold no registers through the spread tests
        const v3 qaL = kSpread == 0 ? qa : v3{s.qgrid.step[0] * inv.x, s.qgrid.step[1] * inv.y, s.qgrid.step[2] * inv.z};
        const v3 qbL = kSpread == 0 ? qb : v3{(s.qgrid.origin[0] - o.x) * inv.x, (s.qgrid.origin[1] - o.y) * inv.y,
                                              (s.qgrid.origin[2] - o.z) * inv.z};
        while (static_cast<unsigned>(ref) < static_cast<unsigned>(kRefDone)) {
            if (kCount) {
                phaseCount(&cnt->innerIters, &cnt->innerLanes);
                if (lanesBelowIn(__ballot(true)) == 0) {
                    cnt->innerIdle += idleLanes;
                    cnt->innerDone += doneLanes;
                }
            }
            const float curLim = cullLimit<kInner>(fminf(bt, shT));
            const bool finite = __ballot(!finiteInv(inv)) == 0;
            const int order = kAny ? s.anyOrder : 0;
            ref = refTree ? innerStep<kInner>(nodeBuf, ref, o, d, inv, curLim, st, cnt, kCount, finite, order)
                          : order == 0 ? innerStepQ<kInner, 0>(qBuf, ldsTop, top, ref, qaL, qbL, curLim, st, cnt, kCount)
                                       : innerStepQ<kInner, 1>(qBuf, ldsTop, top, ref, qaL, qbL, curLim, st, cnt, kCount);
            if (ref < 0 && leaf >= 0) {  // postpone this leaf, keep walking
                leaf = ref;
                ref = popCulled(st, curLim, cull);
            }
            // leave for the leaf phase once fewer than kInnerExit lanes are still looking for a
            // leaf (the rest wait one phase; waiting for the very last costs more)
            if (__popcll(__ballot(leaf >= 0 && static_cast<unsigned>(ref) < static_cast<unsigned>(kRefDone))) < innerExit)
                break;
        }
        // ---- leaves ----
        if constexpr (kSpread != 0) {
        // Wave-uniform: every lane takes part in the spread rounds, holding a leaf or not.
        constexpr uint32_t kNoHitBits = 0x7F800001u;  // a signalling NaN: no arithmetic result has these bits
        while (__ballot(leaf < 0) != 0) {
            const bool holding = leaf < 0;
            int first = 0, nprim = 0;
            float4 a0 = make_float4(0.0F, 0.0F, 0.0F, 0.0F), b0t = a0, c0 = a0;
            if (holding) {
                if (kCount) phaseCount(&cnt->leafIters, &cnt->leafLanes);
                first = leafFirst(leaf);
                nprim = leafCount(leaf);
                const uint32_t off0 = static_cast<uint32_t>(first) * 48u;
                a0 = bload3(triBuf, off0);
                b0t = bload3(triBuf, off0 + 16u);
                c0 = bload3(triBuf, off0 + 32u);
                if (!refTree) {
                    const uint32_t lo = static_cast<uint32_t>(first) * 48u;
                    const float4 b0 = bload4(leafBuf, lo);
                    if (kCount) ++cnt->leaves;
                    if (kCull == kCullExact) {
                        const float4 b1 = bload4(leafBuf, lo + 16u);
                        const float4 b2 = bload4(leafBuf, lo + 32u);
                        float te, ex, ey, ez;
                        if (!slabFiniteAxes(b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, o, inv, &te, &ex, &ey, &ez)) {
                            nprim = 0;
                        } else {
                            const float lim = fminf(bt, shT);
                            if (te > lim && leafKey(b1, b2, te, ex, ey, ez, d, inv) > lim) nprim = 0;
                        }
                    } else {
                        const int2 b1 = bload2i(leafBuf, lo + 16u);
                        float te;
                        const bool in =
                            slabFinite(b0.x, b0.y, b0.z, b0.w, __int_as_float(b1.x), __int_as_float(b1.y), o, inv, &te);
                        if (!in || (cull && te > cullLimit<kCull>(fminf(bt, shT)))) nprim = 0;
                    }
                }
            }
            // this lane's first triangle, tested here
            bool hit = false;
            if (nprim > 0) {
                if (kCount) phaseCount(&cnt->triIters, &cnt->triLanes);
                const uint32_t code = encodePrim(kTriangle, static_cast<uint32_t>(first));
                float t, u, v;
                if (code != src) {
                    if (kCount) ++cnt->tris;
                    if (triTest(a0, b0t, c0, o, d, &t, &u, &v) && !(t < kEpsilon)) {
                        if (kAny) {
                            hit = !(t >= bt);
                        } else if (betterThan(t, code, bt, bcode)) {
                            bt = t;
                            bcode = code;
                        }
                    }
                }
            }
            // the others: slice k = the lanes with a (k+1)-th triangle left (an occluded any-hit lane
            // has none), laid out slice after slice, 64 tests per round
            const uint64_t m1 = __ballot(nprim > 1 && !hit);
            if (m1 != 0) {
                const uint64_t m2 = __ballot(nprim > 2 && !hit), m3 = __ballot(nprim > 3 && !hit);
                const int c1 = __popcll(m1), c12 = c1 + __popcll(m2), total = c12 + __popcll(m3);
                // the owner of every test, by its place in the layout (this wave's LDS table): lane
                // byte-writes, then reads by the same wave (LDS operations of a wave complete in order)
                uint8_t* const owners = spreadOwners + 192 * (threadIdx.x >> 6);
                if (nprim > 1 && !hit) owners[lanesBelowIn(m1)] = static_cast<uint8_t>(lane);
                if (nprim > 2 && !hit) owners[c1 + lanesBelowIn(m2)] = static_cast<uint8_t>(lane);
                if (nprim > 3 && !hit) owners[c12 + lanesBelowIn(m3)] = static_cast<uint8_t>(lane);
                __builtin_amdgcn_wave_barrier();
                bool hit2 = false;
                for (int base = 0; base < total; base += 64) {
                    // tester: test g's slice and owner lane
                    const int g = base + lane;
                    const int tk = g < c1 ? 1 : g < c12 ? 2 : 3;
                    const int own = g < total ? static_cast<int>(owners[g]) : lane;
                    const int srcLane = own << 2;  // ds_bpermute byte address
                    const v3 to{__int_as_float(__builtin_amdgcn_ds_bpermute(srcLane, __float_as_int(o.x))),
                                __int_as_float(__builtin_amdgcn_ds_bpermute(srcLane, __float_as_int(o.y))),
                                __int_as_float(__builtin_amdgcn_ds_bpermute(srcLane, __float_as_int(o.z)))};
                    const v3 td{__int_as_float(__builtin_amdgcn_ds_bpermute(srcLane, __float_as_int(d.x))),
                                __int_as_float(__builtin_amdgcn_ds_bpermute(srcLane, __float_as_int(d.y))),
                                __int_as_float(__builtin_amdgcn_ds_bpermute(srcLane, __float_as_int(d.z)))};
                    const uint32_t tsrc = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(srcLane, static_cast<int>(src)));
                    const int tj = leafFirst(__builtin_amdgcn_ds_bpermute(srcLane, leaf)) + tk;
                    uint32_t tt = kNoHitBits;
                    if (g < total) {
                        if (kCount) phaseCount(&cnt->triIters, &cnt->triLanes);
                        const uint32_t code = encodePrim(kTriangle, static_cast<uint32_t>(tj));
                        if (code != tsrc) {
                            if (kCount) ++cnt->tris;
                            const uint32_t off = static_cast<uint32_t>(tj) * 48u;
                            const float4 ta = bload3(triBuf, off), tb = bload3(triBuf, off + 16u), tc = bload3(triBuf, off + 32u);
                            float t, u, v;
                            if (triTest(ta, tb, tc, to, td, &t, &u, &v) && !(t < kEpsilon)) tt = __float_as_uint(t);
                        }
                    }
                    // owners: the results of their tests in this round, in triangle order
#pragma unroll
                    for (int k = 1; k <= 3; ++k) {
                        const uint64_t mk = k == 1 ? m1 : k == 2 ? m2 : m3;  // (uniform)
                        const int idx = (k == 1 ? 0 : k == 2 ? c1 : c12) + lanesBelowIn(mk);
                        const bool mine = ((mk >> lane) & 1ull) != 0 && idx >= base && idx < base + 64;
                        const uint32_t rt = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute((idx - base) << 2, static_cast<int>(tt)));
                        if (mine && rt != kNoHitBits) {
                            const float t = __uint_as_float(rt);
                            const uint32_t code = encodePrim(kTriangle, static_cast<uint32_t>(leafFirst(leaf) + k));
                            if (kAny) {
                                hit2 = hit2 || !(t >= bt);
                            } else if (betterThan(t, code, bt, bcode)) {
                                bt = t;
                                bcode = code;
                            }
                        }
                    }
                }
                hit = hit || hit2;
                __builtin_amdgcn_wave_barrier();  // (the table is rewritten by the next leaf iteration)
            }
            if (holding) {
                if (kAny && hit) {
                    if (kCount) cnt->occluded += (rayIdx >= 0 && pend == 0) ? 1u : 0u;  // (else counted at the merge)
                    if (rayIdx >= 0 && pend == 0) {
                        q.occ(rayIdx, 1.0F);
                        rayIdx = -1;
                    } else {  // a helper, or an owner waiting for helpers: the merge writes it
                        occ = true;
                    }
                    st.sp = 0;
                    ref = kRefDone;
                    leaf = 0;
                } else {
                    leaf = 0;
                    if (ref < 0) {  // the next node is a leaf too: test it now
                        leaf = ref;
                        ref = popCulled(st, cullLimit<kInner>(fminf(bt, shT)), cull);
                    }
                }
            }
            if (__popcll(__ballot(leaf < 0)) < leafExit) break;
        }
        } else {
        while (leaf < 0) {
            if (kCount) phaseCount(&cnt->leafIters, &cnt->leafLanes);
            const int first = leafFirst(leaf);
            int nprim = leafCount(leaf);
            // the first triangle's loads go out with the leaf box's (one round trip, not two)
            const uint32_t off0 = static_cast<uint32_t>(first) * 48u;
            const float4 a0 = bload3(triBuf, off0), b0t = bload3(triBuf, off0 + 16u), c0 = bload3(triBuf, off0 + 32u);
            if (!refTree) {
                // a walk-tree leaf passed a quantized (outward) box: the reference's own test of
                // its exact box, and the cull against that box's entry, decide (BVH.hpp:357-363)
                const uint32_t lo = static_cast<uint32_t>(first) * 48u;
                const float4 b0 = bload4(leafBuf, lo);
                if (kCount) ++cnt->leaves;
                if (kCull == kCullExact) {
                    const float4 b1 = bload4(leafBuf, lo + 16u);
                    const float4 b2 = bload4(leafBuf, lo + 32u);
                    float te, ex, ey, ez;
                    if (!slabFiniteAxes(b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, o, inv, &te, &ex, &ey, &ez)) {
                        nprim = 0;
                    } else {
                        // certified leaf cull: the key never exceeds the entry, so only a leaf
                        // entered beyond the best needs it; skipped iff every acceptable t of
                        // its triangles exceeds the best (then no tie is possible either)
                        const float lim = fminf(bt, shT);
                        if (te > lim && leafKey(b1, b2, te, ex, ey, ez, d, inv) > lim) nprim = 0;
                    }
                } else {
                    const int2 b1 = bload2i(leafBuf, lo + 16u);
                    float te;
                    const bool in =
                        slabFinite(b0.x, b0.y, b0.z, b0.w, __int_as_float(b1.x), __int_as_float(b1.y), o, inv, &te);
                    if (!in || (cull && te > cullLimit<kCull>(fminf(bt, shT)))) nprim = 0;
                }
            }
            bool hit = false;
            // software-pipelined (kPrefetch): triangle k + 1's loads go out before triangle k's test
            constexpr bool kPrefetch = kAny ? MRT_TRI_PREFETCH_ANY != 0 : MRT_TRI_PREFETCH != 0;
            float4 ca = a0, cb = b0t, cc = c0;
            for (int k = 0; k < nprim; ++k) {
                if (kCount) phaseCount(&cnt->triIters, &cnt->triLanes);
                const int j = first + k;
                float4 ta = ca, tb = cb, tc = cc;
                if constexpr (kPrefetch) {
                    if (k + 1 < nprim) {
                        const uint32_t offn = static_cast<uint32_t>(j + 1) * 48u;
                        ca = bload3(triBuf, offn);
                        cb = bload3(triBuf, offn + 16u);
                        cc = bload3(triBuf, offn + 32u);
                    }
                } else if (k > 0) {
                    const uint32_t off = static_cast<uint32_t>(j) * 48u;
                    ta = bload3(triBuf, off);
                    tb = bload3(triBuf, off + 16u);
                    tc = bload3(triBuf, off + 32u);
                }
                const uint32_t code = encodePrim(kTriangle, static_cast<uint32_t>(j));
                if (code == src) continue;
                float t, u, v;
                if (kCount) ++cnt->tris;
                if (!triTest(ta, tb, tc, o, d, &t, &u, &v)) continue;
                if (t < kEpsilon) continue;
                if (kAny) {
                    if (!(t >= bt)) {
                        hit = true;
                        break;
                    }
                } else if (betterThan(t, code, bt, bcode)) {
                    bt = t;
                    bcode = code;
                }
            }
            if (kAny && hit) {
                if (kCount) cnt->occluded += (rayIdx >= 0 && pend == 0) ? 1u : 0u;  // (else counted at the merge)
                if (rayIdx >= 0 && pend == 0) {
                    q.occ(rayIdx, 1.0F);
                    rayIdx = -1;
                } else {  // a helper, or an owner waiting for helpers: the merge writes it
                    occ = true;
                }
                st.sp = 0;
                ref = kRefDone;
                leaf = 0;
                break;
            }
            leaf = 0;
            if (ref < 0) {  // the next node is a leaf too: test it now
                leaf = ref;
                ref = popCulled(st, cullLimit<kInner>(fminf(bt, shT)), cull);
            }
            // back to the inner phase once fewer than kLeafExit lanes hold a leaf: the others keep
            // theirs (tested first when the leaf phase resumes, so each lane's order is unchanged)
            if (__popcll(__ballot(leaf < 0)) < leafExit) break;
        }
        }
    }
}

// A level's queue arrays (k_trace / k_shadow): rays [0, count) of rOs / rDs, results into out.
template <bool kAny, bool kCount, int kCull, class Stack>
__device__ __forceinline__ void traceWhileWhile(const DScene& s, const float4* __restrict__ rOs,
                                                const float4* __restrict__ rDs, float4* out, const SegMap& map,
                                                int* fetch, Stack& st, TravCount* cnt, const QNode4* ldsTop,
                                                int* tailBest) {
    LevelQueue q(rOs, rDs, out, map, fetch);
    traceWhileWhileQ<kAny, kCount, kCull>(s, q, st, cnt, ldsTop, tailBest);
}

}  // namespace mrt
