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

namespace mrt {

constexpr int kRefDone = 0x7FFFFFFF;  // sentinel: no node (never a valid inner index)

__device__ __forceinline__ int popCulled(TStack& st, float lim, bool cull) {
    while (st.sp > 0) {
        const int2 e = st.pop();
        if (!cull || !(__int_as_float(e.y) > lim)) return e.x;
    }
    return kRefDone;
}

// kAny = false: closest hit -> writes lv.hit;  kAny = true: shadow any-hit -> writes lv.sC.w
template <bool kAny, bool kCount>
__device__ __forceinline__ void traceWhileWhile(const DScene& s, const float4* __restrict__ rOs,
                                                const float4* __restrict__ rDs, float4* out, int count, int* fetch,
                                                TStack& st, TravCount* cnt) {
    const int lane = static_cast<int>(threadIdx.x & 63u);
    const uint64_t lanesBelow = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const GNode* __restrict__ nodes = s.triNodes;
    int rayIdx = -1;
    bool exhausted = false;
    v3 o{0, 0, 0}, d{0, 0, 0}, inv{0, 0, 0};
    uint32_t src = 0;
    Best b{kRayLengthMax, 0.0F, 0.0F, kNoPrim};
    int ref = kRefDone;
    int leaf = 0;  // < 0: a postponed leaf
    while (true) {
        // ---- lanes whose triangle walk is over: lights (closest only), write the result ----
        if (rayIdx >= 0 && ref == kRefDone && leaf >= 0) {
            if (kAny) {
                out[rayIdx].w = 0.0F;
            } else {
                for (int j = 0; j < s.nLights; ++j) {  // Shader.cpp:166-171
                    const float4* l = s.lights + 4 * j;
                    const float4 a4 = l[0];
                    if (__float_as_int(a4.w) != 1) continue;
                    float t, u, v;
                    if (!triTest(a4, l[1], l[2], o, d, &t, &u, &v)) continue;
                    if (t < kEpsilon) continue;
                    const uint32_t code = encodePrim(kLight, static_cast<uint32_t>(j));
                    if (better(t, code, b)) b = Best{t, u, v, code};
                }
                out[rayIdx] = make_float4(b.t, b.u, b.v, bitsf(b.code));
            }
            rayIdx = -1;
        }
        // ---- refill lanes without a ray (one atomic per wave) ----
        const bool need = rayIdx < 0 && !exhausted;
        const uint64_t needMask = __ballot(need);
        if (needMask != 0) {
            const int n = __popcll(needMask);
            const int leader = __ffsll(static_cast<unsigned long long>(needMask)) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(fetch, n);
            base = __shfl(base, leader, 64);
            if (need) {
                rayIdx = base + __popcll(needMask & lanesBelow);
                if (rayIdx >= count) {
                    exhausted = true;
                    rayIdx = -1;
                } else {
                    const float4 o4 = rOs[rayIdx];
                    const float4 d4 = rDs[rayIdx];
                    o = xyz(o4);
                    d = xyz(d4);
                    inv = v3{1.0F / d.x, 1.0F / d.y, 1.0F / d.z};
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
                    if (rayIdx >= 0) {
                        float te;
                        const GRoot& r = s.triRoot;
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
        if (__ballot(rayIdx >= 0) == 0) {
            if (__ballot(!exhausted) == 0) break;
            continue;
        }
        // ---- inner nodes until every active lane holds a postponed leaf ----
        while (static_cast<unsigned>(ref) < static_cast<unsigned>(kRefDone)) {
            const float4* np = reinterpret_cast<const float4*>(nodes + ref);
            const float4 n0 = np[0], n1 = np[1], n2 = np[2];
            const int4 n3 = reinterpret_cast<const int4*>(np)[3];
            if (kCount) cnt->nodes += 2;
            float tl, tr;
            bool hl = slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, o, inv, &tl);
            bool hr = slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, o, inv, &tr);
            const float curLim = b.t + b.t * kCullMargin;
            if (s.cull) {
                hl = hl && !(tl > curLim);
                hr = hr && !(tr > curLim);
            }
            if (hl && hr) {
                int nearRef = n3.x, farRef = n3.y;
                float farT = tr;
                if (s.cull && tr < tl) {
                    nearRef = n3.y;
                    farRef = n3.x;
                    farT = tl;
                }
                st.push(farRef, farT);
                ref = nearRef;
            } else if (hl) {
                ref = n3.x;
            } else if (hr) {
                ref = n3.y;
            } else {
                ref = popCulled(st, curLim, s.cull != 0);
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
            for (int k = 0; k < nprim; ++k) {
                const int j = first + k;
                const uint32_t code = encodePrim(kTriangle, static_cast<uint32_t>(j));
                if (code == src) continue;
                const float4* g = s.triGeom + 3 * j;
                float t, u, v;
                if (kCount) ++cnt->tris;
                if (!triTest(g[0], g[1], g[2], o, d, &t, &u, &v)) continue;
                if (t < kEpsilon) continue;
                if (kAny) {
                    if (!(t >= b.t)) {
                        hit = true;
                        break;
                    }
                } else if (better(t, code, b)) {
                    b = Best{t, u, v, code};
                }
            }
            if (kAny && hit) {
                out[rayIdx].w = 1.0F;
                rayIdx = -1;
                st.sp = 0;
                ref = kRefDone;
                leaf = 0;
                break;
            }
            leaf = 0;
            if (ref < 0) {  // the next node is a leaf too: test it now
                leaf = ref;
                ref = popCulled(st, b.t + b.t * kCullMargin, s.cull != 0);
            }
        }
    }
}

}  // namespace mrt
