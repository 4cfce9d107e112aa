// mrt_trace_ww.hpp - persistent "while-while" triangle-BVH traversal for wave64.
//
// Same reachability, culling and tie rules as traverse<> in mrt_device.hpp (so results are
// identical, tested), organised for SIMD efficiency on CDNA's 64-lane waves:
//   * inner nodes are walked until EVERY active lane has found a leaf (leaves are postponed
//     one at a time), then all lanes test their leaves together: inner-node and leaf code no
//     longer alternate inside one wave iteration;
//   * lanes whose ray has finished take a new ray immediately (one wave-aggregated atomic per
//     refill) instead of idling until the slowest ray of a 64-ray batch is done.
// Planes / spheres (tiny BVHs, empty for OBJ scenes) are tested at ray fetch with the simple
// walker, area lights when the triangle walk ends, in the reference's category order.
#pragma once

#include "mrt_device.hpp"
#include "mrt_kernels.hpp"

namespace mrt {

constexpr int kRefDone = 0x7FFFFFFF;  // sentinel: no node (never a valid inner index)

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
__device__ __forceinline__ uint4 bload4u(BufRes r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// number of set bits of a wave mask below this lane
__device__ __forceinline__ int lanesBelowIn(uint64_t m) {
    return static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
}

__device__ __forceinline__ int popCulled(TStack& st, float lim, bool cull) {
    while (st.sp > 0) {
        const int2 e = st.pop();
        if (!cull || !(__int_as_float(e.y) > lim)) return e.x;
    }
    return kRefDone;
}

// Culling, near-first order and the push of the far child, shared by the node formats.
__device__ __forceinline__ int chooseChildren(bool hl, bool hr, float tl, float tr, int refL, int refR, float lim,
                                              bool cull, TStack& st) {
    if (cull) {
        hl = hl && !(tl > lim);
        hr = hr && !(tr > lim);
    }
    if (hl && hr) {
        int nearRef = refL, farRef = refR;
        float farT = tr;
        if (cull && tr < tl) {
            nearRef = refR;
            farRef = refL;
            farT = tl;
        }
        st.push(farRef, farT);
        return nearRef;
    }
    if (hl) return refL;
    if (hr) return refR;
    return popCulled(st, lim, cull);
}

// kAny = false: closest hit -> writes lv.hit;  kAny = true: shadow any-hit -> writes lv.sC.w
// One BVH2 inner-node visit: returns the next node (near child, or a popped entry).
// top: nodes [0, top) are read from the LDS copy ldsTop (the breadth-first top of the tree)
// finite: wave-uniform, every active lane's 1/d is finite (slabFinite applies)
template <int kTop>
__device__ __forceinline__ int innerStep2(BufRes nodes, const GNode* ldsTop, int top, int ref, v3 o, v3 inv,
                                          float lim, bool cull, TStack& st, TravCount* cnt, bool count, bool finite) {
    float4 n0, n1, n2;
    int2 n3;
    if (kTop > 0 && ref < top) {
        const float4* np = reinterpret_cast<const float4*>(ldsTop + ref);
        n0 = np[0];
        n1 = np[1];
        n2 = np[2];
        n3 = reinterpret_cast<const int2*>(np)[6];
    } else {
        const uint32_t off = static_cast<uint32_t>(ref) * static_cast<uint32_t>(sizeof(GNode));
        n0 = bload4(nodes, off);
        n1 = bload4(nodes, off + 16u);
        n2 = bload4(nodes, off + 32u);
        n3 = bload2i(nodes, off + 48u);  // child refs (the rest is padding)
    }
    if (count) cnt->nodes += 2;
    float tl, tr;
    bool hl, hr;
    if (finite) {
        hl = slabFinite(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, o, inv, &tl);
        hr = slabFinite(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, o, inv, &tr);
    } else {
        hl = slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, o, inv, &tl);
        hr = slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, o, inv, &tr);
    }
    return chooseChildren(hl, hr, tl, tr, n3.x, n3.y, lim, cull, st);
}

// One visit of a compressed node (CNode: 2 loads instead of 4) for waves whose rays all have
// finite 1/d.  The dequantised child boxes contain the exact ones and the finite-1/d slab is
// monotone in the bounds (each t = (bound - o) * inv is a monotone function of the bound, and
// min / max / >= preserve it), so every child whose exact box passes passes here too; a child
// that passes only its enlarged box costs a visit, never a result, because a leaf's triangles
// count only once the leaf's exact box passes (leafReachable) - and a leaf whose exact box
// passes has every ancestor's exact box passing too (they contain it).  Nodes [0, top) are the
// exact LDS copy.
template <int kTop>
__device__ __forceinline__ int innerStepC(BufRes cnodes, const GNode* ldsTop, int top, int ref, v3 o, v3 inv,
                                          float lim, bool cull, TStack& st, TravCount* cnt, bool count) {
    float lx0, ly0, lz0, lx1, ly1, lz1, rx0, ry0, rz0, rx1, ry1, rz1;
    int refL, refR;
    if (kTop > 0 && ref < top) {
        const float4* np = reinterpret_cast<const float4*>(ldsTop + ref);
        const float4 n0 = np[0], n1 = np[1], n2 = np[2];
        const int2 n3 = reinterpret_cast<const int2*>(np)[6];
        lx0 = n0.x; ly0 = n0.y; lz0 = n0.z; lx1 = n0.w; ly1 = n1.x; lz1 = n1.y;
        rx0 = n1.z; ry0 = n1.w; rz0 = n2.x; rx1 = n2.y; ry1 = n2.z; rz1 = n2.w;
        refL = n3.x;
        refR = n3.y;
    } else {
        const uint32_t off = static_cast<uint32_t>(ref) * static_cast<uint32_t>(sizeof(CNode));
        const uint4 a = bload4u(cnodes, off);
        const uint4 b = bload4u(cnodes, off + 16u);
        const float ox = __uint_as_float(a.x), oy = __uint_as_float(a.y), oz = __uint_as_float(a.z);
        const float qx = __uint_as_float((a.w & 0xFFu) << 23);
        const float qy = __uint_as_float(((a.w >> 8) & 0xFFu) << 23);
        const float qz = __uint_as_float(((a.w >> 16) & 0xFFu) << 23);
        auto u8 = [](uint32_t w, int k) { return static_cast<float>((w >> (8 * k)) & 0xFFu); };
        lx0 = fmaf(qx, u8(b.x, 0), ox);
        ly0 = fmaf(qy, u8(b.x, 1), oy);
        lz0 = fmaf(qz, u8(b.x, 2), oz);
        lx1 = fmaf(qx, u8(b.x, 3), ox);
        ly1 = fmaf(qy, u8(b.y, 0), oy);
        lz1 = fmaf(qz, u8(b.y, 1), oz);
        rx0 = fmaf(qx, u8(b.y, 2), ox);
        ry0 = fmaf(qy, u8(b.y, 3), oy);
        rz0 = fmaf(qz, u8(b.z, 0), oz);
        rx1 = fmaf(qx, u8(b.z, 1), ox);
        ry1 = fmaf(qy, u8(b.z, 2), oy);
        rz1 = fmaf(qz, u8(b.z, 3), oz);
        const uint32_t meta = a.w >> 24;
        const int v = static_cast<int>(b.w);
        const int cL = static_cast<int>((meta >> 2) & 3u) + 1, cR = static_cast<int>((meta >> 4) & 3u) + 1;
        const bool lLeaf = (meta & 1u) != 0, rLeaf = (meta & 2u) != 0;
        refL = lLeaf ? leafRef(v, cL) : ref + 1;
        refR = rLeaf ? leafRef(lLeaf ? v + cL : v, cR) : (lLeaf ? ref + 1 : v);
    }
    if (count) cnt->nodes += 2;
    float tl, tr;
    const bool hl = slabFinite(lx0, ly0, lz0, lx1, ly1, lz1, o, inv, &tl);
    const bool hr = slabFinite(rx0, ry0, rz0, rx1, ry1, rz1, o, inv, &tr);
    return chooseChildren(hl, hr, tl, tr, refL, refR, lim, cull, st);
}

// The reference reaches a leaf iff its exact box passes (see innerStepC); finite 1/d only.
__device__ __forceinline__ bool leafReachable(BufRes leafBoxes, int first, v3 o, v3 inv) {
    const uint32_t off = static_cast<uint32_t>(first) * 32u;
    const float4 a = bload4(leafBoxes, off);
    const int2 b = bload2i(leafBoxes, off + 16u);
    float te;
    return slabFinite(a.x, a.y, a.z, a.w, __int_as_float(b.x), __int_as_float(b.y), o, inv, &te);
}

__device__ __forceinline__ void cas(float& ka, int& ra, float& kb, int& rb) {
    if (kb < ka) {
        const float tk = ka;
        ka = kb;
        kb = tk;
        const int tr = ra;
        ra = rb;
        rb = tr;
    }
}

// One 4-wide visit: tests the four child boxes, pushes the hit children far-to-near.
__device__ __forceinline__ int innerStep4(const GNode4* node, v3 o, v3 inv, float lim, bool cull, TStack& st,
                                          TravCount* cnt, bool count) {
    const float4* np = reinterpret_cast<const float4*>(node);
    const float4 mnx = np[0], mny = np[1], mnz = np[2], mxx = np[3], mxy = np[4], mxz = np[5];
    const int4 cr = reinterpret_cast<const int4*>(np)[6];
    if (count) cnt->nodes += (cr.x != kRefEmpty) + (cr.y != kRefEmpty) + (cr.z != kRefEmpty) + (cr.w != kRefEmpty);
    constexpr float kInf = __builtin_huge_valf();
    float t0, t1, t2, t3;
    const bool h0 = cr.x != kRefEmpty && slab(mnx.x, mny.x, mnz.x, mxx.x, mxy.x, mxz.x, o, inv, &t0) && !(cull && t0 > lim);
    const bool h1 = cr.y != kRefEmpty && slab(mnx.y, mny.y, mnz.y, mxx.y, mxy.y, mxz.y, o, inv, &t1) && !(cull && t1 > lim);
    const bool h2 = cr.z != kRefEmpty && slab(mnx.z, mny.z, mnz.z, mxx.z, mxy.z, mxz.z, o, inv, &t2) && !(cull && t2 > lim);
    const bool h3 = cr.w != kRefEmpty && slab(mnx.w, mny.w, mnz.w, mxx.w, mxy.w, mxz.w, o, inv, &t3) && !(cull && t3 > lim);
    const int n = static_cast<int>(h0) + static_cast<int>(h1) + static_cast<int>(h2) + static_cast<int>(h3);
    if (n == 0) return popCulled(st, lim, cull);
    float k0 = h0 ? t0 : kInf, k1 = h1 ? t1 : kInf, k2 = h2 ? t2 : kInf, k3 = h3 ? t3 : kInf;
    int r0 = cr.x, r1 = cr.y, r2 = cr.z, r3 = cr.w;
    if (!h0) r0 = kRefEmpty;
    if (!h1) r1 = kRefEmpty;
    if (!h2) r2 = kRefEmpty;
    if (!h3) r3 = kRefEmpty;
    cas(k0, r0, k1, r1);  // 4-element sorting network, misses (inf) sink to the end
    cas(k2, r2, k3, r3);
    cas(k0, r0, k2, r2);
    cas(k1, r1, k3, r3);
    cas(k1, r1, k2, r2);
    if (n > 3) st.push(r3, k3);
    if (n > 2) st.push(r2, k2);
    if (n > 1) st.push(r1, k1);
    return r0;
}


// Position of the r-th (0-based) set bit of m (m must have more than r set bits).
__device__ __forceinline__ int nthSetBit(uint64_t m, int r) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint64_t low = m & ((1ull << w) - 1ull);
        const int c = __popcll(low);
        if (r >= c) {
            r -= c;
            m >>= w;
            pos += w;
        }
    }
    return pos;
}

// Takes the bottom entry of a non-empty stack (the subtree nearest the root: the largest piece
// of work to hand over); the top entry moves into its place.  Entry k lives in the global
// spill area (gofs + k) while k < sp - depth, else in LDS slot k % depth.
__device__ __forceinline__ int2 takeBottom(TStack& st) {
    if (st.sp == 1) return st.pop();
    const int2 top = st.pop();
    int2 b;
    if (st.sp > st.depth) {
        b = st.gbase[st.gofs];
        st.gbase[st.gofs] = top;
    } else {
        b = st.lds[0];
        st.lds[0] = top;
    }
    return b;
}

// kAssist ("tail assist"): once the queue is empty, lanes without a ray help the rays still
// walking in their wave.  A walking lane hands the bottom entry of its stack (a whole subtree)
// to an idle lane, which walks it with a copy of the ray and the owner's best hit so far; when
// the helper's walk ends its result is merged into the owner lane with the same total order
// (betterThan) - closest hit and occlusion do not depend on the order in which subtrees are
// walked, so results are identical.  The last rays of a launch (up to ~8x the mean walk) no
// longer run on one lane each while the rest of the GPU idles.
// kTrim: a wave that moves on from a drained cursor reads the next cursor before it takes from
// it (a load instead of an atomic on an address every wave of the launch hits at the end).
// kComp: compressed nodes (innerStepC) for all-finite waves, and a leaf's triangles count only
// once its exact box passes (lanes with finite 1/d; the others only ever take exact steps).
template <bool kAny, bool kCount, int kWide, int kRefill, int kShards, int kTop, bool kFastSlab, bool kAssist = false,
          bool kTrim = false, bool kComp = false, bool kOcc = false>
__device__ __forceinline__ void traceWhileWhile(const DScene& s, const float4* __restrict__ rOs,
                                                const float4* __restrict__ rDs, float4* out, int count, int* fetch,
                                                TStack& st, TravCount* cnt, const GNode* ldsTop,
                                                const int* __restrict__ order) {
    const int top = kTop > 0 ? min(kTop, s.triTop) : 0;
    const BufRes nodeBuf = bufferOf(s.triNodes);
    const BufRes triBuf = bufferOf(s.triGeom);
    constexpr bool kC = kComp && !kCount;  // counting builds count the exact walk
    const BufRes cnodeBuf = bufferOf(kC ? static_cast<const void*>(s.triCNodes) : static_cast<const void*>(s.triNodes));
    const BufRes leafBuf = bufferOf(kC ? static_cast<const void*>(s.leafBoxes) : static_cast<const void*>(s.triNodes));
    const int lane = static_cast<int>(threadIdx.x & 63u);
    int rayIdx = -1;
    bool exhausted = false;
    v3 o{0, 0, 0}, d{0, 0, 0}, inv{0, 0, 0};
    uint32_t src = 0;
    // closest hit so far: t and primitive code only; u, v are recomputed for the winner at
    // the end (same inputs -> same bits), which keeps two registers out of the walk
    float bt = kRayLengthMax;
    uint32_t bcode = kNoPrim;
    int ref = kRefDone;
    int leaf = 0;  // < 0: a postponed leaf
    int seg = static_cast<int>(blockIdx.x % kShards);  // wave-uniform cursor state
    int segsLeft = kShards;
    constexpr bool kAs = kAssist && !kCount;  // counting builds keep the canonical per-ray walk
    int helpOf = -1;     // kAs: the owner lane of the ray this lane helps with (-1: not helping)
    int nHelp = 0;       // kAs, owner: helpers still walking parts of this lane's ray
    bool occl = false;   // kAs && kAny: occlusion found (by this lane or a helper)
    uint32_t t0 = 0;     // kAs: fetch time of this lane's ray (100 MHz ticks)
    // kOcc (shadow rays): the triangle that occluded this lane's previous shadow ray is tested
    // first.  A hit with eps <= t < distance in a leaf whose exact box passes is one the walk
    // would find (the reference reaches that leaf: every ancestor's box contains it and the
    // finite-1/d slab test is monotone in the bounds), and any hit makes the answer "occluded"
    // (BVH.hpp:350-351), so the walk is skipped; otherwise the ray walks as usual.
    constexpr bool kO = kOcc && kAny && !kCount && !kAs;
    const BufRes occBuf = bufferOf(kO ? static_cast<const void*>(s.occBoxes) : static_cast<const void*>(s.triNodes));
    int lastOcc = -1;
    while (true) {
        if (kAs) {
            // ---- helpers whose walk is over: merge into the owner lane (same total order) ----
            uint64_t hm = __ballot(helpOf >= 0 && ref == kRefDone && leaf >= 0);
            while (hm != 0) {
                const int h = __ffsll(static_cast<unsigned long long>(hm)) - 1;
                const int ho = __builtin_amdgcn_readlane(helpOf, h);
                const float ht = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bt), h));
                const uint32_t hc = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(bcode), h));
                const int hocc = __builtin_amdgcn_readlane(static_cast<int>(occl), h);
                if (lane == ho) {
                    if (kAny) {
                        occl = occl || hocc != 0;
                    } else if (betterThan(ht, hc, bt, bcode)) {
                        bt = ht;
                        bcode = hc;
                    }
                    --nHelp;
                }
                hm &= hm - 1ull;
            }
            if (helpOf >= 0 && ref == kRefDone && leaf >= 0) {
                helpOf = -1;
                occl = false;
            }
            if (__ballot(helpOf >= 0) != 0) {
                // helpers follow the owner: a closer hit tightens their culling; an occluded
                // shadow ray needs no more walking
                const int ol = helpOf >= 0 ? helpOf : lane;
                const float obt = __shfl(bt, ol, 64);
                const uint32_t oc = static_cast<uint32_t>(__shfl(static_cast<int>(bcode), ol, 64));
                const int oo = __shfl(static_cast<int>(occl), ol, 64);
                if (helpOf >= 0) {
                    if (kAny) {
                        if (oo != 0) {
                            st.sp = 0;
                            ref = kRefDone;
                            leaf = 0;
                        }
                    } else if (betterThan(obt, oc, bt, bcode)) {
                        bt = obt;
                        bcode = oc;
                    }
                }
            }
        }
        // ---- lanes whose triangle walk is over: lights (closest only), write the result ----
        if (rayIdx >= 0 && ref == kRefDone && leaf >= 0 && (!kAs || nHelp == 0)) {
            if (kCount) cnt->rayMax = max(cnt->rayMax, cnt->nodes - cnt->rayStart);
            if (kAs) cnt->ticksMax = max(cnt->ticksMax, static_cast<uint32_t>(wall_clock64()) - t0);
            if (kAny) {
                out[rayIdx].w = (kAs && occl) ? 1.0F : 0.0F;
                occl = false;
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
                out[rayIdx] = make_float4(bt, u, v, bitsf(bcode));
            }
            rayIdx = -1;
        }
        // ---- refill lanes without a ray (one atomic per wave) ----
        bool need = rayIdx < 0 && !exhausted;
        uint64_t needMask = __ballot(need);
        // refill only once enough lanes are idle (fewer, larger fetches), or when none is busy
        if (kRefill > 1 && __popcll(needMask) < kRefill && __ballot(rayIdx >= 0 || helpOf >= 0) != 0) {
            need = false;
            needMask = 0;
        }
        if (needMask != 0) {
            int got = -1;
            if (kShards == 1) {
                const int n = __popcll(needMask);
                const int leader = __ffsll(static_cast<unsigned long long>(needMask)) - 1;
                int base = 0;
                if (lane == leader) base = atomicAdd(fetch, n);
                base = __shfl(base, leader, 64);
                got = base + lanesBelowIn(needMask);
                if (got >= count) got = -1;
            } else {
                // per-XCD-group cursors over contiguous ray ranges; an empty range is left
                // for the next one (speed only: any placement gives the same results)
                uint64_t pending = needMask;
                while (pending != 0 && segsLeft > 0) {
                    const int n = __popcll(pending);
                    const int leader = __ffsll(static_cast<unsigned long long>(pending)) - 1;
                    const int segStart = static_cast<int>((static_cast<long long>(count) * seg) / kShards);
                    const int segEnd = static_cast<int>((static_cast<long long>(count) * (seg + 1)) / kShards);
                    int base = 0;
                    if (lane == leader) {
                        int* cur = fetch + seg * kFetchStride;
                        if (kTrim && segsLeft < kShards &&
                            __hip_atomic_load(cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= segEnd - segStart) {
                            base = segEnd - segStart;
                        } else {
                            base = atomicAdd(cur, n);
                        }
                    }
                    base = __shfl(base, leader, 64);
                    const bool mine = ((pending >> lane) & 1ull) != 0;
                    if (mine) {
                        const int idx = segStart + base + lanesBelowIn(pending);
                        if (idx < segEnd) got = idx;
                    }
                    pending = __ballot(mine && got < 0);
                    if (pending != 0) {
                        seg = (seg + 1) % kShards;
                        --segsLeft;
                    }
                }
            }
            if (need) {
                rayIdx = (got >= 0 && order != nullptr) ? order[got] : got;
                if (kCount) cnt->rayStart = cnt->nodes;
                if (kAs) t0 = static_cast<uint32_t>(wall_clock64());
                if (rayIdx < 0) {
                    exhausted = true;
                } else {
                    const float4 o4 = rOs[rayIdx];
                    const float4 d4 = rDs[rayIdx];
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
                            out[rayIdx].w = 1.0F;
                            rayIdx = -1;
                        }
                    } else {
                        src = fbits(d4.w);
                        b = Best{kRayLengthMax, 0.0F, 0.0F, kNoPrim};
                        traverse<kPlane, false>(s, s.planeNodes, s.planeRoot, o, d, inv, src, &b, st, cnt);
                        traverse<kSphere, false>(s, s.sphereNodes, s.sphereRoot, o, d, inv, src, &b, st, cnt);
                    }
                    bt = b.t;
                    bcode = b.code;
                    if (kO && rayIdx >= 0 && lastOcc >= 0 && finiteInv(inv)) {
                        const uint32_t code = encodePrim(kTriangle, static_cast<uint32_t>(lastOcc));
                        const uint32_t off = static_cast<uint32_t>(lastOcc) * 48u;
                        float t, u, v;
                        if (code != src &&
                            triTest(bload3(triBuf, off), bload3(triBuf, off + 16u), bload3(triBuf, off + 32u), o, d, &t,
                                    &u, &v) &&
                            !(t < kEpsilon) && !(t >= bt) && leafReachable(occBuf, lastOcc, o, inv)) {
                            out[rayIdx].w = 1.0F;
                            rayIdx = -1;
                        }
                    }
                    if (rayIdx >= 0) {
                        float te;
                        const GRoot& r = kWide == 4 ? s.triRoot4 : s.triRoot;
                        if (r.count > 0 &&
                            slab(r.bmin[0], r.bmin[1], r.bmin[2], r.bmax[0], r.bmax[1], r.bmax[2], o, inv, &te)) {
                            ref = r.ref;
                            if (ref < 0) {  // the root is a leaf
                                leaf = ref;
                                ref = kRefDone;
                            }
                        }
                    }
                }
            }
        }
        if (kAs) {
            // ---- tail assist: idle lanes (queue empty) take a subtree of a walking lane ----
            const bool idle = rayIdx < 0 && helpOf < 0 && exhausted;
            const uint64_t idleMask = __ballot(idle);
            const bool canGive = (rayIdx >= 0 || helpOf >= 0) && ref != kRefDone && st.sp > 0 && !(kAny && occl);
            const uint64_t giveMask = __ballot(canGive);
            if (idleMask != 0 && giveMask != 0) {
                const int nPairs = min(__popcll(idleMask), __popcll(giveMask));
                const bool gives = canGive && lanesBelowIn(giveMask) < nPairs;
                if (gives) ++cnt->assists;
                int2 e = make_int2(kRefDone, 0);
                if (gives) e = takeBottom(st);
                const int ir = lanesBelowIn(idleMask);
                const bool takes = idle && ir < nPairs;
                const int from = takes ? nthSetBit(giveMask, ir) : lane;
                const int ownerOf = helpOf >= 0 ? helpOf : lane;
                const int eRef = __shfl(e.x, from, 64);
                const float eT = __int_as_float(__shfl(e.y, from, 64));
                const int nOwner = __shfl(ownerOf, from, 64);
                const v3 no{__shfl(o.x, from, 64), __shfl(o.y, from, 64), __shfl(o.z, from, 64)};
                const v3 nd{__shfl(d.x, from, 64), __shfl(d.y, from, 64), __shfl(d.z, from, 64)};
                const v3 ni{__shfl(inv.x, from, 64), __shfl(inv.y, from, 64), __shfl(inv.z, from, 64)};
                const uint32_t nsrc = static_cast<uint32_t>(__shfl(static_cast<int>(src), from, 64));
                const float nbt = __shfl(bt, from, 64);
                const uint32_t nbc = static_cast<uint32_t>(__shfl(static_cast<int>(bcode), from, 64));
                // owners count their new helpers (one per giving lane of their ray)
                uint64_t gm = __ballot(gives);
                while (gm != 0) {
                    const int g = __ffsll(static_cast<unsigned long long>(gm)) - 1;
                    if (lane == __builtin_amdgcn_readlane(ownerOf, g)) ++nHelp;
                    gm &= gm - 1ull;
                }
                if (takes) {
                    helpOf = nOwner;
                    o = no;
                    d = nd;
                    inv = ni;
                    src = nsrc;
                    bt = nbt;
                    bcode = nbc;
                    occl = false;
                    st.sp = 0;
                    leaf = 0;
                    ref = (s.cull != 0 && eT > bt + bt * kCullMargin) ? kRefDone : eRef;  // as popCulled
                    if (ref < 0) {  // a leaf
                        leaf = ref;
                        ref = kRefDone;
                    }
                }
            }
        }
        if (__ballot(rayIdx >= 0 || (kAs && helpOf >= 0)) == 0) {
            if (__ballot(!exhausted) == 0) break;
            continue;
        }
        // ---- inner nodes until every active lane holds a postponed leaf ----
        while (static_cast<unsigned>(ref) < static_cast<unsigned>(kRefDone)) {
            const float curLim = bt + bt * kCullMargin;
            if (kWide == 4) {
                ref = innerStep4(s.triNodes4 + ref, o, inv, curLim, s.cull != 0, st, cnt, kCount);
            } else {
                const bool finite = kFastSlab && __ballot(!finiteInv(inv)) == 0;
                if (kC && finite) {
                    ref = innerStepC<kTop>(cnodeBuf, ldsTop, top, ref, o, inv, curLim, s.cull != 0, st, cnt, kCount);
                } else {
                    ref = innerStep2<kTop>(nodeBuf, ldsTop, top, ref, o, inv, curLim, s.cull != 0, st, cnt, kCount,
                                           finite);
                }
            }
            if (ref < 0 && leaf >= 0) {  // postpone this leaf, keep walking
                leaf = ref;
                ref = popCulled(st, curLim, s.cull != 0);
            }
            if (__ballot(leaf >= 0 && static_cast<unsigned>(ref) < static_cast<unsigned>(kRefDone)) == 0) break;
        }
        // ---- leaves ----
        while (leaf < 0) {
            const int first = leafFirst(leaf), nprim = leafCount(leaf);
            bool hit = false;
            // kC: whether the reference reaches this leaf, looked up at its first would-be hit
            // (-1 not yet known; lanes with a non-finite 1/d walked exact nodes only)
            int reach = (kC && finiteInv(inv)) ? -1 : 1;
            for (int k = 0; k < nprim; ++k) {
                const int j = first + k;
                const uint32_t code = encodePrim(kTriangle, static_cast<uint32_t>(j));
                if (code == src) continue;
                const uint32_t off = static_cast<uint32_t>(j) * 48u;
                float t, u, v;
                if (kCount) ++cnt->tris;
                if (!triTest(bload3(triBuf, off), bload3(triBuf, off + 16u), bload3(triBuf, off + 32u), o, d, &t, &u, &v))
                    continue;
                if (t < kEpsilon) continue;
                const bool cand = kAny ? !(t >= bt) : betterThan(t, code, bt, bcode);
                if (!cand) continue;
                if (kC && reach < 0) reach = leafReachable(leafBuf, first, o, inv) ? 1 : 0;
                if (kC && reach == 0) break;  // the reference never tests this leaf's triangles
                if (kAny) {
                    if (kO) lastOcc = j;
                    hit = true;
                    break;
                }
                bt = t;
                bcode = code;
            }
            if (kAny && hit) {
                if (kAs) {
                    occl = true;  // written when the helpers of this ray are done
                } else {
                    out[rayIdx].w = 1.0F;
                    rayIdx = -1;
                }
                st.sp = 0;
                ref = kRefDone;
                leaf = 0;
                break;
            }
            leaf = 0;
            if (ref < 0) {  // the next node is a leaf too: test it now
                leaf = ref;
                ref = popCulled(st, bt + bt * kCullMargin, s.cull != 0);
            }
        }
    }
}

}  // namespace mrt
