// mrt_trace_packet.hpp - wave-coherent ("packet") closest-hit walk for coherent rays on wave64.
//
// The camera rays of a wave are 16 neighbouring pixels x 4 samples (k_raygen's queue order), so
// their walks over the quantized 4-wide tree nearly coincide.  Here the 64 rays of a wave share
// ONE traversal: a wave-uniform stack of node references in LDS, each node fetched once per wave
// through the scalar cache (uniform addresses in the constant address space become s_load), and
// a child entered when ANY walking lane's ray passes its quantized box (a ballot).  Every lane
// still decides its own leaves exactly as the per-lane walk does (traceWhileWhile): its own test
// of the reference leaf box, the certified leaf cull of the exact mode, and its own triangle
// tests (triangle records again scalar loads).  The packet visits a superset of each lane's
// inner nodes.  Its lanes test exactly the leaves they would test alone PROVIDED every quantized
// box on the path to a leaf holds that leaf's exact box as the slab test computes it, for every
// lane's ray (the Quantizer's one-grid-step margin): then a lane reaches a
// leaf in the packet iff its own walk would, and the exact leaf-box test and the certified leaf key
// decide as they do alone.  betterThan is a total order, so each lane's closest hit is the per-lane
// walk's, bit for bit (tested: full frames, random rays, and coherent 64-ray bundles grazing
// leaf-box corners, edges and faces in tests/test_full_frame.py).  No lane diverges inside the
// loop, so VALU lanes stay busy on coherent rays.
// Cull modes 0 (none) and 3 (exact) only: neither culls an inner node.
#pragma once

#include <type_traits>

#include "mrt_trace_ww.hpp"

namespace mrt {

// Scalar (SGPR) loads: dwords read through the constant address space at a wave-uniform address
typedef __attribute__((address_space(4))) const uint32_t ConstU32;
__device__ __forceinline__ int4 sload4i(ConstU32* p) {
    return make_int4(static_cast<int>(p[0]), static_cast<int>(p[1]), static_cast<int>(p[2]), static_cast<int>(p[3]));
}
__device__ __forceinline__ float4 sload4f(ConstU32* p) {
    return make_float4(__uint_as_float(p[0]), __uint_as_float(p[1]), __uint_as_float(p[2]), __uint_as_float(p[3]));
}

// Keeps scalar-loaded values in SGPRs at this point: every load issued before the first pin is
// waited for once, there (an empty asm that reads them).
__device__ __forceinline__ void pinSgprs(float4 v) { asm volatile("" ::"s"(v.x), "s"(v.y), "s"(v.z), "s"(v.w)); }
__device__ __forceinline__ void pinSgprs(int4 v) { asm volatile("" ::"s"(v.x), "s"(v.y), "s"(v.z), "s"(v.w)); }

// One triangle of the leaf being tested by the packet: A, AB, AC (triGeom's xyz), wave-uniform.
struct PacketTri {
    float4 a, ab, ac;
    __device__ __forceinline__ void pin() const {
        asm volatile("" ::"s"(a.x), "s"(a.y), "s"(a.z), "s"(ab.x), "s"(ab.y), "s"(ab.z));
        asm volatile("" ::"s"(ac.x), "s"(ac.y), "s"(ac.z));
    }
    // this lane's test (the per-lane walk's: triTest, the t >= epsilon rule, betterThan)
    template <bool kCount>
    __device__ __forceinline__ void test(uint32_t code, bool lane, uint32_t src, v3 o, v3 d, float* bt, uint32_t* bcode,
                                         TravCount* cnt) const {
        if (!lane || code == src) return;
        if (kCount) ++cnt->tris;
        float t, u, v;
        if (triTest(a, ab, ac, o, d, &t, &u, &v) && !(t < kEpsilon) && betterThan(t, code, *bt, *bcode)) {
            *bt = t;
            *bcode = code;
        }
    }
};
__device__ __forceinline__ PacketTri loadPacketTri(ConstU32* tg, int j) {
    return PacketTri{sload4f(tg + 12 * j), sload4f(tg + 12 * j + 4), sload4f(tg + 12 * j + 8)};
}

// A node reference made wave-uniform (it is, by construction; this tells the compiler).
__device__ __forceinline__ int uniformInt(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Closest hit of camera rays: rOs / rDs -> out = (t, u, v, primitive code).  (The any-hit form
// for the level-1 shadow rays was built, exact and slower: DESIGN.md section 3.1.)
// post(i, valid, o4, d4, hit): called by every lane of the wave after each packet (the fused
// level-1 shading of k_trace_packet_shade; a no-op otherwise).
struct NoPost {
    __device__ __forceinline__ void operator()(int, bool, float4, float4, float4) const {}
};
// rays(i, &o4, &d4): ray i (the fused kernel generates camera rays; otherwise rOs / rDs are read)
struct NoRays {
    __device__ __forceinline__ void operator()(int, float4*, float4*) const {}
};
// next(): the first ray index of the wave's next packet (wave-uniform); >= count ends the walk
#ifndef MRT_PACKET_SEGMENTS
#define MRT_PACKET_SEGMENTS 1
#endif
#if MRT_PACKET_SEGMENTS
// the level queue's packets over kWalkShards cursors (kFetchStride ints apart; each serving its
// interleaved chunks, mrt_trace_ww.hpp), a workgroup starting on its XCD group's cursor (blockIdx %
// 8) and trying walkSegments() of them: the exhausted-queue polls spread over 8 addresses
struct PacketFetch {
    int* fetch;
    int count;
    int seg = static_cast<int>(blockIdx.x % kWalkShards);
    int segsLeft = walkSegments();
    __device__ __forceinline__ int next() {
        const int packets = (count + 63) >> 6;
        while (segsLeft > 0) {
            const int first = static_cast<int>((static_cast<long long>(packets) * seg) / kWalkShards);
            const int last = static_cast<int>((static_cast<long long>(packets) * (seg + 1)) / kWalkShards);
            int p = 0;
            if ((threadIdx.x & 63u) == 0) p = atomicAdd(fetch + seg * kFetchStride, 1);
            p = __shfl(p, 0, 64);
#if MRT_SEG_INTERLEAVE
            // the walk cursors' interleaved chunks (mrt_trace_ww.hpp), in 64-ray packets
            (void)first;
            (void)last;
            const int q = interleavedIndex(p, seg, segChunkShift(packets, kSegChunkLog - 6));
            if (q < packets) return q << 6;
#else
            if (first + p < last) return (first + p) << 6;
#endif
            seg = (seg + 1) % kWalkShards;
            --segsLeft;
        }
        return count;
    }
};
#else
struct PacketFetch {  // the level queue: 64 rays per atomic on one cursor
    int* fetch;
    int count;
    __device__ __forceinline__ int next() const {
        int base = 0;
        if ((threadIdx.x & 63u) == 0) base = atomicAdd(fetch, 64);
        return __shfl(base, 0, 64);
    }
};
#endif
struct OnePacket {  // one packet: rays [0, count) (the tile kernel's camera rays)
    int done = 0;
    __device__ __forceinline__ int next() { return done++ == 0 ? 0 : 64; }
};
template <bool kCount, int kCull, class Stack, class Post = NoPost, class Rays = NoRays, class Fetch = PacketFetch>
__device__ __forceinline__ void tracePacketF(const DScene& s, const float4* __restrict__ rOs,
                                             const float4* __restrict__ rDs, float4* out, int count, Fetch fetch,
                                             Stack& st, TravCount* cnt, int* waveStack, Post post = Post(),
                                             Rays rays = Rays()) {
    static_assert(kCull == kCullNone || kCull == kCullExact, "packet walk: cull modes 0 and 3");
    ConstU32* const qnf = (ConstU32*)(s.triQNodesF);  // NOLINT: address-space casts
    ConstU32* const tg = (ConstU32*)(s.triGeom);      // NOLINT
    ConstU32* const lb = (ConstU32*)(s.leafBoxes);    // NOLINT
    const int lane = static_cast<int>(threadIdx.x & 63u);
    while (true) {
        const int base = uniformInt(fetch.next());
        if (base >= count) break;
        const int i = base + lane;
        const bool valid = i < count;
        v3 o{0, 0, 0}, d{1, 1, 1};
        uint32_t src = 0;
        float4 o4 = make_float4(0.0F, 0.0F, 0.0F, 0.0F), d4 = o4;
        if (valid) {
            if constexpr (std::is_same<Rays, NoRays>::value) {
                o4 = rOs[i];
                d4 = rDs[i];
            } else {
                rays(i, &o4, &d4);
            }
            o = xyz(o4);
            d = xyz(d4);
            src = fbits(d4.w);
        }
        const v3 inv{1.0F / d.x, 1.0F / d.y, 1.0F / d.z};
        // lanes outside the quantized grid's bound (a zero direction component, ...) take the
        // per-lane reference walk after the packet (rare; divergent)
        const bool packed = valid && quantOK(s, o, inv);
        Best b{kRayLengthMax, 0.0F, 0.0F, kNoPrim};
        if (packed) {
            traverse<kPlane, false>(s, s.planeNodes, s.planeRoot, o, d, inv, src, &b, st, cnt);
            traverse<kSphere, false>(s, s.sphereNodes, s.sphereRoot, o, d, inv, src, &b, st, cnt);
        }
        float bt = b.t;
        uint32_t bcode = b.code;
        const v3 qa{s.qgrid.step[0] * inv.x, s.qgrid.step[1] * inv.y, s.qgrid.step[2] * inv.z};
        const v3 qb{(s.qgrid.origin[0] - o.x) * inv.x, (s.qgrid.origin[1] - o.y) * inv.y,
                    (s.qgrid.origin[2] - o.z) * inv.z};
        const GRoot& r = s.triRoot;
        float te;
        const bool walking =
            packed && r.count > 0 && slab(r.bmin[0], r.bmin[1], r.bmin[2], r.bmax[0], r.bmax[1], r.bmax[2], o, inv, &te);
        const uint64_t walkers = __ballot(walking);
        int ref = walkers != 0 ? r.ref : kRefDone;  // uniform
        int sp = 0;                                 // uniform
        // the lane whose entries order the children: the first walking one
        const int lead = walkers != 0 ? __ffsll(static_cast<unsigned long long>(walkers)) - 1 : 0;
        while (ref != kRefDone) {
            if (ref >= 0) {  // ---- inner node: four children, entered on any lane's hit ----
                // the node's float grid indices (DScene::triQNodesF): one scalar round trip
                if (kCount && lane == 0) ++cnt->innerIters;  // per wave: 128 B through the scalar cache
                float4 nf[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) nf[j] = sload4f(qnf + 32 * ref + 4 * j);
#pragma unroll
                for (int j = 0; j < 8; ++j) pinSgprs(nf[j]);
                const auto fw = [&](int k) -> float {  // word k (a compile-time constant after unrolling)
                    const float4 v = nf[k >> 2];
                    const int c = k & 3;
                    return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
                };
                uint32_t key[kWalkWidth];
                int rf[kWalkWidth];
                int n = 0;
#pragma unroll
                for (int c = 0; c < kWalkWidth; ++c) {
                    rf[c] = __float_as_int(fw(24 + c));
                    const bool used = rf[c] != kEmptyChild;  // uniform
                    // the per-lane walk's planes bit for bit (float(q) is exact); every lane
                    // computes, the walking ones count
                    float t;
                    const bool h = qslab(fw(6 * c), fw(6 * c + 1), fw(6 * c + 2), fw(6 * c + 3), fw(6 * c + 4),
                                         fw(6 * c + 5), qa, qb, &t);
                    if (kCount && walking && used) cnt->nodes += 1u;
                    const uint64_t m = __builtin_amdgcn_ballot_w64(h) & walkers;  // (no short circuit:
                    const bool any = (m != 0u) & used;                              // straight-line code)
                    // order: the lead lane's entry (entries are >= 0: their bits sort as unsigned
                    // integers); children it misses go last
                    const uint32_t k = static_cast<uint32_t>(
                        __builtin_amdgcn_readlane(static_cast<int>(h ? __float_as_uint(t) : 0x7F800000u), lead));
                    key[c] = any ? k : 0xFFFFFFFFu;
                }
                // children entered (counted on the uniform keys: scalar code)
#pragma unroll
                for (int c = 0; c < kWalkWidth; ++c) {  // (integer form: no lane-mask booleans)
                    const uint32_t x = ~key[c];
                    n += static_cast<int>((x | (0u - x)) >> 31);
                }
                if (n == 0) {
                    ref = sp > 0 ? uniformInt(waveStack[--sp]) : kRefDone;
                    continue;
                }
                // ascending sort of the (key, reference) pairs (uniform values: scalar code)
                const auto cex = [&](int a, int c) {
                    if (key[c] < key[a]) {
                        const uint32_t tk = key[a];
                        key[a] = key[c];
                        key[c] = tk;
                        const int tr = rf[a];
                        rf[a] = rf[c];
                        rf[c] = tr;
                    }
                };
                cex(0, 1);
                cex(2, 3);
                cex(0, 2);
                cex(1, 3);
                cex(1, 2);
#pragma unroll
                for (int c = kWalkWidth - 1; c >= 1; --c)
                    if (c < n) {
                        if (lane == 0) waveStack[sp] = rf[c];
                        ++sp;
                    }
                ref = rf[0];
                continue;
            }
            // ---- a leaf: each walking lane tests the reference box, then its triangles ----
            // The leaf record and the leaf's first two triangles are fetched in one scalar round
            // trip (pinned before any use, so the compiler cannot sink a load behind a branch and
            // pay a second trip), the remaining triangles two per trip.
            const int first = leafFirst(ref);
            const int nprim = leafCount(ref);
            const int lastTri = r.count - 1;
            const float4 b0 = sload4f(lb + 12 * first), b1 = sload4f(lb + 12 * first + 4), b2 = sload4f(lb + 12 * first + 8);
            PacketTri tri0 = loadPacketTri(tg, first), tri1 = loadPacketTri(tg, min(first + 1, lastTri));
            if (kCount && lane == 0) {  // per wave: the 48-B leaf record and two 48-B triangle records
                ++cnt->leafIters;
                cnt->triIters += 2u;
            }
            pinSgprs(b0);
            pinSgprs(b1);
            pinSgprs(b2);
            tri0.pin();
            tri1.pin();
            bool test = false;
            if (walking) {
                if (kCount) ++cnt->leaves;
                float tl, ex, ey, ez;
                test = slabFiniteAxes(b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, o, inv, &tl, &ex, &ey, &ez);
                // the exact mode's certified leaf cull (mrt_trace_ww.hpp leafKey)
                if (kCull == kCullExact && test && tl > bt && leafKey(b1, b2, tl, ex, ey, ez, d, inv) > bt) test = false;
            }
            if (__ballot(test) != 0) {
                for (int k = 0; k < nprim; k += 2) {
                    if (k > 0) {
                        if (kCount && lane == 0) cnt->triIters += 2u;
                        tri0 = loadPacketTri(tg, first + k);
                        tri1 = loadPacketTri(tg, min(first + k + 1, lastTri));
                        tri0.pin();
                        tri1.pin();
                    }
                    tri0.test<kCount>(encodePrim(kTriangle, static_cast<uint32_t>(first + k)), test, src, o, d, &bt, &bcode, cnt);
                    if (k + 1 < nprim)
                        tri1.test<kCount>(encodePrim(kTriangle, static_cast<uint32_t>(first + k + 1)), test, src, o, d, &bt,
                                          &bcode, cnt);
                }
            }
            ref = sp > 0 ? uniformInt(waveStack[--sp]) : kRefDone;
        }
        float4 hit = make_float4(0.0F, 0.0F, 0.0F, 0.0F);
        if (valid) {
            if (!packed) {
                const Best f = closestHit(s, o, d, src, st, cnt);
                hit = make_float4(f.t, f.u, f.v, bitsf(f.code));
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
                float u = b.u, v = b.v, t;  // planes / spheres keep their (0, 0)
                const uint32_t kind = primKind(bcode);
                if (kind == kTriangle || kind == kLight) {  // the winner's u, v: same inputs, same bits
                    const float4* g = kind == kTriangle ? s.triGeom + 3 * primIndex(bcode) : s.lights + 4 * primIndex(bcode);
                    (void)triTest(g[0], g[1], g[2], o, d, &t, &u, &v);
                } else {
                    u = 0.0F;
                    v = 0.0F;
                }
                hit = make_float4(bt, u, v, bitsf(bcode));
            }
            // (the fused level-1 kernel shades the hit right here: nothing reads it from memory)
            if constexpr (std::is_same<Post, NoPost>::value) out[i] = hit;
            if (kCount) ++cnt->rays;
        }
        post(i, valid, o4, d4, hit);
    }
}

template <bool kCount, int kCull, class Stack, class Post = NoPost, class Rays = NoRays>
__device__ __forceinline__ void tracePacket(const DScene& s, const float4* __restrict__ rOs,
                                            const float4* __restrict__ rDs, float4* out, int count, int* fetch,
                                            Stack& st, TravCount* cnt, int* waveStack, Post post = Post(),
                                            Rays rays = Rays()) {
    tracePacketF<kCount, kCull>(s, rOs, rDs, out, count, PacketFetch{fetch, count}, st, cnt, waveStack, post, rays);
}

}  // namespace mrt
