// mrt_kernels.hip - the wavefront render pipeline for gfx950 (MI355X).
//
// One "path" = one (pixel, sample) camera ray and the ray tree the shader grows from it.
// A frame is processed level by level (level == ray depth, Ray.hpp depth_):
//
//   raygen (level 1)                       Renderer.cpp:130-141, Perspective.cpp:16-28
//   for L = 1 .. maxDepth+1:
//     trace    closest hit of level L      Shader.cpp:86-111, BVH.hpp:327-384
//     shade    vertex records, shadow rays, child rays of level L+1 (wave-aggregated
//              compaction: one atomic per wave)           Whitted.cpp / PathTracer.cpp
//     shadow   any-hit of the shadow rays  Shader.cpp:132-158
//   for L = maxDepth+1 .. 1:
//     resolve  bottom-up radiance of every vertex, in the reference's float-op order
//   accumulate incrementalAvg per pixel, sample by sample   Utils.cpp:66-90
//
// Evaluating the ray tree bottom-up (instead of forward throughput) keeps every float
// operation in the order of the recursive reference, which is what makes the Whitted
// Cornell image bit-exact.
#include "mrt_kernels.hpp"
#include "mrt_trace_ww.hpp"
#include "mrt_trace_packet.hpp"

#include <algorithm>
#include <atomic>
#include <utility>

namespace mrt {

// ---------------------------------------------------------------------------------------
// wave helpers (wave64)
__device__ __forceinline__ int laneId() { return static_cast<int>(threadIdx.x & 63u); }

__device__ __forceinline__ int waveExclusiveScan(int v, int* total) {
    const int lane = laneId();
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    *total = __shfl(x, 63, 64);
    return x - v;
}

// Allocates n slots per lane from *counter with ONE atomic per wave; every lane of the
// wave must call it (n = 0 for idle lanes).
__device__ __forceinline__ int waveAlloc(int* counter, int n) {
    int total;
    const int excl = waveExclusiveScan(n, &total);
    int base = 0;
    if (laneId() == 63 && total > 0) base = atomicAdd(counter, total);
    base = __shfl(base, 63, 64);
    return base + excl;
}

// Allocates nLo / nHi slots per thread from a pair of adjacent int counters {lo, hi} with
// ONE 64-bit atomic per block (same-address atomics serialise at the memory side: per-wave
// allocation made them the shading kernel's limiter).  Every thread of the block must call
// it; lds holds 2 x (waves + 1) entries, alternated by the caller's parity.
__device__ __forceinline__ void blockAllocPair(unsigned long long* pair, int nLo, int nHi, int* baseLo, int* baseHi,
                                               unsigned long long* lds, int parity) {
    constexpr int kWaves = kBlock / 64;
    const int lane = laneId();
    const int wave = static_cast<int>(threadIdx.x >> 6);
    const unsigned long long v =
        (static_cast<unsigned long long>(static_cast<unsigned>(nHi)) << 32) | static_cast<unsigned>(nLo);
    unsigned long long x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    unsigned long long* buf = lds + parity * (kWaves + 1);
    if (lane == 63) buf[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long sum = 0;
        for (int w = 0; w < kWaves; ++w) {
            const unsigned long long t = buf[w];
            buf[w] = sum;
            sum += t;
        }
        buf[kWaves] = sum != 0 ? atomicAdd(pair, sum) : 0ull;
    }
    __syncthreads();
    const unsigned long long e = buf[kWaves] + buf[wave] + (x - v);
    *baseLo = static_cast<int>(static_cast<unsigned>(e & 0xFFFFFFFFull));
    *baseHi = static_cast<int>(static_cast<unsigned>(e >> 32));
}

// ---------------------------------------------------------------------------------------
// pixel mapping: path p -> (pixel slot, sample); slot -> (x, y) through the unit table
__device__ __forceinline__ void slotToXY(const PixelMap& m, int slot, int* x, int* y) {
    int lo = 0, hi = m.nUnits - 1;
    while (lo < hi) {  // last unit whose prefix <= slot
        const int mid = (lo + hi + 1) >> 1;
        if (m.prefix[mid] <= slot) lo = mid; else hi = mid - 1;
    }
    const int4 r = m.rect[lo];
    const int off = slot - m.prefix[lo];
    *x = r.x + off / r.w;  // column-major inside the unit: 8 rows per column
    *y = r.y + off % r.w;
}
// rect.z = unit width (columns), rect.w = unit height (rows)

// Camera ray of path p (Renderer.cpp:108-111, 131-140 with Perspective / Orthographic::generateRay):
// origin (w = path key bits), direction (w = kNoPrim: no source primitive).
__device__ __forceinline__ void cameraRay(const RaygenArgs& a, int p, float4* o4, float4* d4) {
    const int slot = a.slotBase + p / a.spp;
    const int s = p % a.spp;
    int x, y;
    slotToXY(a.map, slot, &x, &y);
    const uint32_t pixelIndex = static_cast<uint32_t>(y * a.width + x);
    const uint32_t key = pathKey(pixelIndex, static_cast<uint32_t>(a.sampleBase + s));
    // Renderer.cpp:108-111, 131-140
    const float invW = 1.0F / static_cast<float>(a.width);
    const float invH = 1.0F / static_cast<float>(a.height);
    const float pixW = 0.5F / static_cast<float>(a.width);
    const float pixH = 0.5F / static_cast<float>(a.height);
    const float u = static_cast<float>(x) * invW;
    const float v = static_cast<float>(y) * invH;
    float r1 = a.constJitter, r2 = a.constJitter;  // Constant(value) (Constant.cpp:9-11)
    if (a.tableJitter != 0) {  // StaticHaltonSeq: the two draws of the pixel sampler, one 8-byte read
        const float2 j = a.jitter[sampleBlock(key, 0u)];
        r1 = j.x;
        r2 = j.y;
    }
    const float devU = (r1 - 0.5F) * 2.0F * pixW;
    const float devV = (r2 - 0.5F) * 2.0F * pixH;
    const GCamera& c = a.cam;
    v3 origin, dir;
    if (c.kind == 1) {  // Orthographic.cpp:15-24 (hFov / vFov hold the half sizes)
        const float rf = (u - 0.5F) * c.hFov;
        const v3 right = c.right * rf + c.right * devU;
        const float uf = (0.5F - v) * c.vFov;
        const v3 up = c.up * uf + c.up * devV;
        origin = (c.position + right) + up;
        dir = c.direction;
    } else {  // Perspective.cpp:16-28
        const float rf = fastArcTan(c.hFov * (u - 0.5F)) + devU;
        const v3 right = c.right * rf;
        const float uf = fastArcTan(c.vFov * (0.5F - v)) + devV;
        const v3 up = c.up * uf;
        const v3 dest = ((c.position + c.direction) + right) + up;
        origin = c.position;
        dir = normalize(dest - c.position);
    }
    *o4 = make_float4(origin.x, origin.y, origin.z, bitsf(key));
    *d4 = make_float4(dir.x, dir.y, dir.z, bitsf(kNoPrim));
}

__global__ __launch_bounds__(256) void k_raygen(RaygenArgs a, Level lv, int* counters) {
    const int p = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (p == 0) denseCounts(counters, 1, false, a.nPaths, lv.segCap);
    if (p >= a.nPaths) return;
    float4 o4, d4;
    cameraRay(a, p, &o4, &d4);
    lv.rO[p] = o4;
    lv.rD[p] = d4;
    lv.tree[p] = 1u;
}

// ---------------------------------------------------------------------------------------
// Trace kernels.  Two walks with identical results (tested):
//   variant 0: per-wave 64-ray batches, if-if walk (closestHit / anyHit of mrt_device.hpp) -
//              the plain restatement of BVH.hpp:327-384, kept as the in-kernel reference;
//   variant 1: the persistent while-while walk of mrt_trace_ww.hpp (default).
constexpr int kWalkThreads = 256;

template <bool kCount>
__device__ __forceinline__ void reduceCounts(const TravCount& cnt, unsigned long long* stats, int nodesStat,
                                             int trisStat, int leavesStat) {
    unsigned long long n = cnt.nodes, t = cnt.tris, l = cnt.leaves;
    for (int off = 32; off > 0; off >>= 1) {
        n += __shfl_down(n, off, 64);
        t += __shfl_down(t, off, 64);
        l += __shfl_down(l, off, 64);
    }
    if (laneId() == 0) {
        atomicAdd(stats + nodesStat, n);
        atomicAdd(stats + trisStat, t);
        atomicAdd(stats + leavesStat, l);
    }
}

// counting builds: the walk phases' wave iterations and active lanes (kind 0 closest, 1 any hit)
__device__ __forceinline__ void reducePhases(const TravCount& cnt, unsigned long long* stats, int kind) {
    const uint32_t v[6] = {cnt.innerIters, cnt.innerLanes, cnt.leafIters, cnt.leafLanes, cnt.triIters, cnt.triLanes};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        unsigned long long x = v[k];
        for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
        if (laneId() == 0 && x != 0) atomicAdd(stats + kStatPhases + 6 * kind + k, x);
    }
    const uint32_t w[2] = {cnt.innerIdle, cnt.innerDone};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        unsigned long long x = w[k];
        for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
        if (laneId() == 0 && x != 0) atomicAdd(stats + kStatPhases + 12 + 2 * kind + k, x);
    }
}

// counting builds: this wave's entry of the wave log (kWaveLogWaves)
__device__ __forceinline__ void waveLog(const TravCount& cnt, unsigned long long* stats, int kind, int level,
                                        unsigned long long t0) {
    unsigned long long n = cnt.nodes, r = cnt.rays;
    for (int off = 32; off > 0; off >>= 1) {
        n += __shfl_down(n, off, 64);
        r += __shfl_down(r, off, 64);
    }
    const int wave = static_cast<int>(blockIdx.x * (kWalkThreads / 64) + threadIdx.x / 64);
    if (laneId() == 0 && wave < kWaveLogWaves && level < kMaxLevels) {
        unsigned long long* e = stats + kNumStats + ((static_cast<size_t>(kind) * kMaxLevels + level) * kWaveLogWaves + wave) * 4;
        e[0] = t0;
        e[1] = __builtin_amdgcn_s_memrealtime();
        e[2] = r;
        e[3] = n;
    }
}

// A walk's traversal stack: the cull modes pop against each entry's key (TStack); the others
// store references only (RefStack: twice the entries in the same LDS)
template <int kCull>
__device__ __forceinline__ auto makeWalkStack(int2* ldsStack, int2* gstack, int gdepth) {
    if constexpr (kCull == kCullFast || kCull == kCullCertified)
        return makeKeyStack<kWalkThreads>(ldsStack, gstack, gdepth);
    else
        return makeRefStack<kWalkThreads>(ldsStack, gstack, gdepth);
}

// Waves per SIMD of the per-lane walks.  Round 5: 6, whose 80 VGPRs hold
// the triangle loop's prefetch of the next triangle (MRT_TRI_PREFETCH, mrt_trace_ww.hpp); 7 waves
// (72 VGPRs) without it measured 3 % slower, 6 waves without it the same as 7.
#ifndef MRT_WALK_WAVES
#define MRT_WALK_WAVES 6
#endif
#ifndef MRT_SHADOW_WAVES
#define MRT_SHADOW_WAVES MRT_WALK_WAVES
#endif
template <bool kCount, int kVariant, int kCull>
__global__ __launch_bounds__(kWalkThreads, MRT_WALK_WAVES) void k_trace(DScene s, Level lv, int* counters, int level,
                                                            int2* gstack, int gdepth, unsigned long long* stats) {
    __shared__ int2 ldsStack[kWalkStack * kWalkThreads];
    auto st = makeWalkStack<kCull>(ldsStack, gstack, gdepth);
    const unsigned long long t0 = kCount ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const SegMap map = segMap(counters, level, false, lv.segCap);
    int* fetch = counters + kCntFetchShards + level * kMaxFetchShards * kFetchStride;
    TravCount cnt{0u, 0u};
    if (kVariant == 1) {
        __shared__ QNode4 ldsTop[kWalkTop];
        __shared__ int tailBest[kWalkThreads];
        stageTop<kWalkThreads>(s, ldsTop);
        traceWhileWhile<false, kCount, kCull>(s, lv.rO, lv.rD, lv.hit, map, fetch, st, &cnt, ldsTop, tailBest);
    }
    while (kVariant == 0) {
        int base = 0;
        if (laneId() == 0) base = atomicAdd(fetch, 64);
        base = __shfl(base, 0, 64);
        if (base >= map.total()) break;
        const int v = base + laneId();
        if (v < map.total()) {
            const int i = map.phys(v);
            const float4 o4 = lv.rO[i];
            const float4 d4 = lv.rD[i];
            const Best b = closestHit(s, xyz(o4), xyz(d4), fbits(d4.w), st, &cnt);
            lv.hit[i] = make_float4(b.t, b.u, b.v, bitsf(b.code));
        }
    }
    if (kCount) {
        reduceCounts<kCount>(cnt, stats, kStatNodes, kStatTris, kStatLeaves);
        reduceCounts<kCount>(cnt, stats, kStatLevelNodes + level - 1, kStatLevelTris + level - 1, kStatLevelLeaves + level - 1);
        reducePhases(cnt, stats, 0);
        atomicMax(stats + kStatMaxNodesRay, static_cast<unsigned long long>(cnt.rayMax));
        waveLog(cnt, stats, 0, level, t0);
    }
}

// Camera rays generated where they are walked (round 6, tuning key 33): cameraRay (k_raygen's
// function) per lane at the start of each packet, and the records k_shade reads stored from there,
// so that k_raygen's launch and the walk's reads of its records are gone.
struct PacketRaysStore {
    const RaygenArgs* a;
    Level lv;
    __device__ __forceinline__ void operator()(int i, float4* o4, float4* d4) const {
        cameraRay(*a, i, o4, d4);
        if (a->storeRays != 0) {  // (else k_shade regenerates them)
            lv.rO[i] = *o4;
            lv.rD[i] = *d4;
            lv.tree[i] = 1u;
        }
    }
};

// Level-1 (camera) rays in cull modes 0 and 3: the wave-coherent walk (mrt_trace_packet.hpp).
// kGen: the walk generates the camera rays (PacketRaysStore) instead of reading k_raygen's.
// (7 waves per SIMD with kGen: at 8 its 64 VGPRs spilled 12 B; the packet walk measured the same
// at 6, 7 and 8, section 3.1 of DESIGN.md)
template <bool kCount, int kCull, bool kGen>
__global__ __launch_bounds__(kWalkThreads, kGen ? 7 : 8) void k_trace_packet(DScene s, Level lv, int* counters, int level,
                                                                   int2* gstack, int gdepth, unsigned long long* stats,
                                                                   RaygenArgs ra) {
    __shared__ int2 ldsStack[kWalkStack * kWalkThreads];  // per-lane fallback walks only
    __shared__ int waveStacks[kWalkThreads / 64][kPacketStack];
    auto st = makeWalkStack<kCull>(ldsStack, gstack, gdepth);
    const unsigned long long t0 = kCount ? __builtin_amdgcn_s_memrealtime() : 0ull;
    if (kGen && blockIdx.x == 0 && threadIdx.x == 0) denseCounts(counters, level, false, ra.nPaths, lv.segCap);  // (k_raygen's)
    // (level 1 is dense: [0, count))
    const int count = kGen ? min(ra.nPaths, lv.cap) : segMap(counters, level, false, lv.segCap).total();
    int* fetch = counters + kCntFetchShards + level * kMaxFetchShards * kFetchStride;
    TravCount cnt{0u, 0u};
    if constexpr (kGen)
        tracePacket<kCount, kCull>(s, lv.rO, lv.rD, lv.hit, count, fetch, st, &cnt, waveStacks[threadIdx.x / 64], NoPost(),
                                   PacketRaysStore{&ra, lv});
    else
        tracePacket<kCount, kCull>(s, lv.rO, lv.rD, lv.hit, count, fetch, st, &cnt, waveStacks[threadIdx.x / 64]);
    if (kCount) {
        reduceCounts<kCount>(cnt, stats, kStatNodes, kStatTris, kStatLeaves);
        reduceCounts<kCount>(cnt, stats, kStatLevelNodes + level - 1, kStatLevelTris + level - 1, kStatLevelLeaves + level - 1);
        // the packet's own per-wave records (its per-lane fallback walks count only per lane, above)
        const uint32_t w[3] = {cnt.innerIters, cnt.leafIters, cnt.triIters};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            unsigned long long x = w[k];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
            if (laneId() == 0 && x != 0) atomicAdd(stats + kStatPacket + k, x);
        }
        waveLog(cnt, stats, 0, level, t0);
    }
}

template <bool kCount, int kVariant, int kCull>
__global__ __launch_bounds__(kWalkThreads, MRT_SHADOW_WAVES) void k_shadow(DScene s, Level lv, int* counters, int level,
                                                             int2* gstack, int gdepth, unsigned long long* stats) {
    __shared__ int2 ldsStack[kWalkStack * kWalkThreads];
    auto st = makeWalkStack<kCull>(ldsStack, gstack, gdepth);
    const unsigned long long t0 = kCount ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const SegMap map = segMap(counters, level, true, lv.shadowSegCap);
    int* fetch = counters + kCntFetchShards + (kMaxLevels + level) * kMaxFetchShards * kFetchStride;
    TravCount cnt{0u, 0u};
    if (kVariant == 1) {
        __shared__ QNode4 ldsTop[kWalkTop];
        __shared__ int tailBest[kWalkThreads];
        stageTop<kWalkThreads>(s, ldsTop);
        traceWhileWhile<true, kCount, kCull>(s, lv.sO, lv.sD, lv.sC, map, fetch, st, &cnt, ldsTop, tailBest);
    }
    while (kVariant == 0) {
        int base = 0;
        if (laneId() == 0) base = atomicAdd(fetch, 64);
        base = __shfl(base, 0, 64);
        if (base >= map.total()) break;
        const int v = base + laneId();
        if (v < map.total()) {
            const int i = map.phys(v);
            const float4 o4 = lv.sO[i];
            const float4 d4 = lv.sD[i];
            const bool occ = anyHit(s, xyz(o4), xyz(d4), fbits(o4.w), d4.w, st, &cnt);
            lv.sC[i].w = occ ? 1.0F : 0.0F;
        }
    }
    if (kCount) {
        reduceCounts<kCount>(cnt, stats, kStatNodesShadow, kStatTrisShadow, kStatLeavesShadow);
        reducePhases(cnt, stats, 1);
        unsigned long long occl = cnt.occluded;
        for (int off = 32; off > 0; off >>= 1) occl += __shfl_down(occl, off, 64);
        if (laneId() == 0) atomicAdd(stats + kStatOccluded, occl);
        waveLog(cnt, stats, 1, level, t0);
    }
}

// Closest hit (kAny false: lv.rO / rD -> lv.hit) or shadow test (true: lv.sO / sD -> lv.sC.w)
// without the BVH: Naive (accelerator 1) walks every primitive, RegularGrid (2) the 3D-DDA of
// gridWalk; any other id except 3 builds no accelerator in the reference, so only the area
// lights can be hit.
template <bool kAny>
__global__ __launch_bounds__(256) void k_trace_other(DScene s, Level lv, int* counters, int level) {
    const SegMap map = segMap(counters, level, kAny, kAny ? lv.shadowSegCap : lv.segCap);
    for (int v = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); v < map.total();
         v += static_cast<int>(gridDim.x * blockDim.x)) {
        const int i = map.phys(v);
        const float4 o4 = kAny ? lv.sO[i] : lv.rO[i];
        const float4 d4 = kAny ? lv.sD[i] : lv.rD[i];
        const v3 o = xyz(o4), d = xyz(d4);
        const uint32_t src = kAny ? fbits(o4.w) : fbits(d4.w);
        Best b{kAny ? d4.w : kRayLengthMax, 0.0F, 0.0F, kNoPrim};
        bool occluded = false;
        if (s.accel == kAccNaive) {
            occluded = naiveWalk<kAny>(s, o, d, src, &b);
        } else if (s.accel == kAccGrid) {  // Shader.cpp:97-101, 142-146: planes, spheres, triangles
            occluded = gridWalk<kPlane, kAny>(s, s.planeGrid, o, d, src, &b) ||
                       gridWalk<kSphere, kAny>(s, s.sphereGrid, o, d, src, &b) ||
                       gridWalk<kTriangle, kAny>(s, s.triGrid, o, d, src, &b);
        }
        if (kAny) {
            lv.sC[i].w = occluded ? 1.0F : 0.0F;
            continue;
        }
        for (int j = 0; j < s.nLights; ++j) {  // Shader.cpp:166-171
            const float4* l = s.lights + 4 * j;
            const float4 a4 = l[0];
            if (__float_as_int(a4.w) != 1) continue;
            float t, u, v;
            if (!triTest(a4, l[1], l[2], o, d, &t, &u, &v)) continue;
            if (t < kEpsilon) continue;
            const uint32_t code = encodePrim(kLight, static_cast<uint32_t>(j));
            if (betterThan(t, code, b.t, b.code)) b = Best{t, u, v, code};
        }
        lv.hit[i] = make_float4(b.t, b.u, b.v, bitsf(b.code));
    }
}

// ---------------------------------------------------------------------------------------
struct HitGeom {
    v3 P, N;
    uint32_t src;  // primitive the child rays start from (spheres: none, Sphere.cpp:77)
};

__device__ __forceinline__ HitGeom hitGeometry(const DScene& s, v3 o, v3 d, float4 h) {
    const uint32_t code = fbits(h.w);
    const uint32_t kind = primKind(code);
    const uint32_t j = primIndex(code);
    HitGeom g;
    g.P = o + d * h.x;  // Triangle.cpp:99, Plane.cpp:62, Sphere.cpp:71
    g.src = code;
    if (kind == kTriangle) {
        const float4 head = s.triHead[j];
        const v3 nA = xyz(head);
        v3 nB = nA, nC = nA;  // a flat triangle's normals are nA's bits
        if ((__float_as_int(head.w) & 1) == 0) {
            nB = xyz(s.triShade[3 * j + 1]);
            nC = xyz(s.triShade[3 * j + 2]);
        }
        const float w = 1.0F - h.y - h.z;  // Triangle.cpp:96-97
        g.N = normalize(nA * w + nB * h.y + nC * h.z);
    } else if (kind == kPlane) {
        g.N = xyz(s.planes[2 * j]);
    } else {  // sphere
        g.N = normalize(g.P - xyz(s.spheres[2 * j]));
        g.src = kNoPrim;
    }
    return g;
}

__device__ __forceinline__ int hitMaterial(const DScene& s, uint32_t code) {
    const uint32_t kind = primKind(code);
    const uint32_t j = primIndex(code);
    if (kind == kTriangle) return (__float_as_int(s.triHead[j].w) >> 1) - 1;
    if (kind == kPlane) return __float_as_int(s.planes[2 * j].w);
    return __float_as_int(s.spheres[2 * j + 1].x);
}

// Texture::loadColor (Texture.cpp:37-48): the nearest texel, no wrapping (coordinates are in
// [0, 1)); the first three bytes from the texel on (a 1- or 2-channel texture reads into the next
// texel, as the reference does; the last texel is clamped where the reference reads past the end).
__device__ __forceinline__ v3 loadColor(const DScene& s, int tex, float tx, float ty) {
    const int4 ti = s.texInfo[tex];
    const int32_t u = static_cast<int32_t>(tx * static_cast<float>(ti.x));
    const int32_t v = static_cast<int32_t>(ty * static_cast<float>(ti.y));
    uint32_t index = static_cast<uint32_t>(v * ti.x * ti.z + u * ti.z);
    const uint32_t size = static_cast<uint32_t>(ti.x * ti.y * ti.z);
    index = min(index, size >= 3u ? size - 3u : 0u);
    const uint8_t* p = s.texels + ti.w + index;
    return v3{static_cast<float>(p[0]) / 255.0F, static_cast<float>(p[1]) / 255.0F, static_cast<float>(p[2]) / 255.0F};
}

// Shader::rayTrace (Shader.cpp:112-120): a hit on a textured material with texture coordinates
// >= 0 overwrites that material's Kd with the texel.  The reference's Kd_ is shared by every hit
// on the material and read by reference in the shaders, so a shade() that traces a child first
// and reads Kd afterwards sees the last texel written in the child's subtree; k_resolve replays
// that from the per-vertex records this function fills.  Returns (texel, material index) or w = -1.
__device__ __forceinline__ float4 textureWrite(const DScene& s, float4 h) {
    const float4 none = make_float4(0.0F, 0.0F, 0.0F, -1.0F);
    const uint32_t code = fbits(h.w);
    if (primKind(code) != kTriangle) return none;
    const uint32_t j = primIndex(code);
    const int mat = __float_as_int(s.triShade[3 * j].w);
    if (mat < 0) return none;
    const int tex = __float_as_int(s.mats[4 * mat + 1].w);
    if (tex < 0) return none;
    const float4 a = s.triTex[2 * j], b = s.triTex[2 * j + 1];
    const float w = 1.0F - h.y - h.z;  // Triangle.cpp:96-98: tA * w + tB * u + tC * v
    const float tx = (a.x * w + a.z * h.y) + b.x * h.z;
    const float ty = (a.y * w + a.w * h.y) + b.y * h.z;
    if (!(tx >= 0.0F && ty >= 0.0F)) return none;
    const v3 c = loadColor(s, tex, tx, ty);
    return make_float4(c.x, c.y, c.z, static_cast<float>(mat));
}

// Shader::getCosineSampleHemisphere (Shader.cpp:188-216).  cos(phi), sin(phi) with
// phi = 2 pi r1 come from the per-entry table of the platform's cosf / sinf (DScene::trig), so
// the bounce direction has the reference's bits.
__device__ __forceinline__ v3 cosineHemisphere(v3 n, float cphi, float sphi, float r2) {
    const float cosTheta = sqrtf(r2);
    v3 u = fabsf(n.x) > 0.1F ? v3{0.0F, 1.0F, 0.0F} : v3{1.0F, 0.0F, 0.0F};
    u = normalize(cross(u, n));
    const v3 v = cross(n, u);
    const v3 dir = (u * (cphi * cosTheta) + v * (sphi * cosTheta)) + n * sqrtf(1.0F - r2);
    return normalize(dir);
}

// Shader.cpp:231 / PathTracer.cpp:55: the light a sample picks
__device__ __forceinline__ uint32_t lightChoice(const DScene& s, float pick) {
    return static_cast<uint32_t>(floorf(pick * static_cast<float>(s.nLights) * 0.99999F));
}

// Light sample i of a shading point (Whitted.cpp:41-53, PathTracer.cpp:53-67):
// returns false when cos <= 0 (no shadow ray is built).
// pick / r / q: the three table draws of this sample (light choice, area-light point)
// lights: DScene::lights, or k_shade's LDS copy of it
__device__ __forceinline__ bool lightSample(const DScene& s, const HitGeom& g, float pick, float r, float q,
                                           v3* dirOut, float* distOut, v3* contribOut, const float4* lights) {
    const uint32_t chosen = lightChoice(s, pick);
    const float4* l = lights + 4 * chosen;
    const float4 a4 = l[0];
    v3 pos;
    if (__float_as_int(a4.w) == 1) {  // AreaLight::getPosition (AreaLight.cpp:17-26)
        if (r + q >= 1.0F) {
            r = 1.0F - r;
            q = 1.0F - q;
        }
        pos = (xyz(a4) + r * xyz(l[1])) + q * xyz(l[2]);
    } else {
        pos = xyz(a4);
    }
    v3 toLight = pos - g.P;
    const float dist = length(toLight);
    toLight = normalize(toLight);
    const float cosNl = dot(g.N, toLight);
    if (!(cosNl > 0.0F)) return false;
    *dirOut = toLight;
    *distOut = dist;
    *contribOut = xyz(l[3]) * cosNl;
    return true;
}

// One shading vertex (Whitted.cpp:13-93, PathTracer.cpp:22-142), split in two halves so the
// caller can allocate queue slots for all lanes in between: shadePrepare reads the hit and
// decides the shadow and child rays, shadeEmit writes them and the vertex record.
struct ShadeState {
    HitGeom g;
    v3 d;
    float ior;
    int mat;
    uint32_t key, tc;
    bool terminal, direct, wantD, wantS, wantT, ok0;
    float4 leaf;  // terminal: the vertex's final radiance (Le), w = hit-a-light flag
    v3 ld0, lc0;  // light sample 0 (kept in registers)
    float dist0, hcos, hsin, hemi2;
    int nShadow, nChild;
    v3 dir0;     // direction of the first child (computed before the slots are allocated)
};

// kw: textureWrite of this hit (w >= 0: the material's Kd is that texel when shade() runs)
// mats / lights: DScene::mats / lights, or k_shade's LDS copies of them
template <int kShader>
__device__ __forceinline__ ShadeState shadePrepare(const DScene& s, float4 o4, float4 d4, float4 h, uint32_t tc,
                                                   int level, const ShadeArgs& a, float4 kw, const float4* mats,
                                                   const float4* lights) {
    ShadeState v{};
    v.terminal = true;
    v.leaf = make_float4(0.0F, 0.0F, 0.0F, 0.0F);
    v.ior = 1.0F;
    v.mat = -1;
    v.key = fbits(o4.w);
    v.tc = tc;
    v.d = xyz(d4);
    if (level > a.maxDepth) return v;  // the depth cap below, taken before the gathers
    // issue every table gather of this vertex at once: their latencies overlap
    // purposes 0-5 of this vertex's block from the compact per-block copy (DScene::vertexDraws)
    const uint32_t blk = sampleBlock(v.key, tc);
    const float4 d0 = s.vertexDraws[2 * blk], d1 = s.vertexDraws[2 * blk + 1];
    const float rr = d0.x;
    v.hcos = d0.y;  // cos, sin of 2 pi r1
    v.hsin = d0.z;
    v.hemi2 = d0.w;
    const float pick0 = d1.x, lr0 = d1.y, lq0 = d1.z;
    const uint32_t code = fbits(h.w);
    const uint32_t kind = primKind(code);
    // Shader.cpp:122: shade only if hit; Whitted.cpp:14-17 / PathTracer.cpp:25-28: depth cap
    if (kind == kMiss || level > a.maxDepth) return v;
    v3 Le, Kd{0, 0, 0}, Ks{0, 0, 0}, Kt{0, 0, 0};
    if (kind == kLight) {
        Le = xyz(lights[4 * primIndex(code) + 3]);
    } else {
        v.mat = hitMaterial(s, code);
        const float4* m = mats + 4 * v.mat;
        const float4 le4 = m[0];
        Le = xyz(le4);
        v.ior = le4.w;
        Kd = kw.w >= 0.0F ? xyz(kw) : xyz(m[1]);
        Ks = xyz(m[2]);
        Kt = xyz(m[3]);
    }
    if (hasPositive(Le)) {  // Whitted.cpp:19-24
        v.leaf = make_float4(Le.x, Le.y, Le.z, 1.0F);
        return v;
    }
    v.terminal = false;
    v.g = hitGeometry(s, xyz(o4), v.d, h);
    v.direct = hasPositive(Kd) && s.nLights > 0;
    if (v.direct) {
        v.ok0 = lightSample(s, v.g, pick0, lr0, lq0, &v.ld0, &v.dist0, &v.lc0, lights);
        v.nShadow = static_cast<int>(v.ok0);
        for (int k = 1; k < a.samplesLight; ++k) {
            v3 ld, lc;
            float dist;
            if (lightSample(s, v.g, s.tables[sampleIndex(v.key, tc, purposeLightPick(k))].x,
                            s.tables[sampleIndex(v.key, tc, purposeLightR(k))].y,
                            s.tables[sampleIndex(v.key, tc, purposeLightS(k))].y, &ld, &dist, &lc, lights))
                ++v.nShadow;
        }
    }
    if (kShader == kShaderPathTracer && hasPositive(Kd)) {  // PathTracer.cpp:89
        v.wantD = level <= kRayDepthMin || rr > 0.5F;
    }
    v.wantS = hasPositive(Ks);
    v.wantT = hasPositive(Kt);
    v.nChild = static_cast<int>(v.wantD) + static_cast<int>(v.wantS) + static_cast<int>(v.wantT);
    return v;
}

// Writes vertex i's shadow rays (level lv, from shadowBase) and children (level nx, from
// childBase) and its record.  Slots past a queue's capacity set the overflow flag (the frame is
// then redone in smaller passes).  deadNext: level + 1 is the depth-capped last level, whose
// rays are counted (the reference constructs them) but never traced, shaded or read, so their
// payloads are not written and their directions not computed.
// shadowEnd / childEnd: the end of the queue segments the bases lie in (slots from there on overflow)
__device__ __forceinline__ void shadeEmit(const DScene& s, const ShadeState& v, int i, const Level& lv, const Level& nx,
                                          int shadowBase, int childBase, int shadowEnd, int childEnd, int* counters,
                                          const ShadeArgs& a, bool deadNext, const float4* lights) {
    if (v.terminal) {
        lv.res[i] = v.leaf;
        lv.vtx[i] = make_int4(-1, 0, 0, 0);
        return;
    }
    // shadow rays (Whitted.cpp:53, PathTracer.cpp:67)
    int written = 0;
    if (v.direct) {
        for (int k = 0; k < a.samplesLight; ++k) {
            v3 ld = v.ld0, lc = v.lc0;
            float dist = v.dist0;
            if (k == 0) {
                if (!v.ok0) continue;
            } else if (!lightSample(s, v.g, s.tables[sampleIndex(v.key, v.tc, purposeLightPick(k))].x,
                                    s.tables[sampleIndex(v.key, v.tc, purposeLightR(k))].y,
                                    s.tables[sampleIndex(v.key, v.tc, purposeLightS(k))].y, &ld, &dist, &lc, lights)) {
                continue;
            }
            const int j = shadowBase + written;
            ++written;
            if (j < shadowEnd) {
                lv.sO[j] = make_float4(v.g.P.x, v.g.P.y, v.g.P.z, bitsf(v.g.src));
                lv.sD[j] = make_float4(ld.x, ld.y, ld.z, dist);
                lv.sC[j] = make_float4(lc.x, lc.y, lc.z, 0.0F);
            } else {
                atomicOr(counters + kCntOverflow, 1);
            }
        }
    }
    // child rays: diffuse (PathTracer.cpp:90-91), specular (:118-120), transmission (:129-131),
    // stored consecutively from childBase
    if (!deadNext) {
        int c = childBase;
        auto emit = [&](v3 dir, uint32_t slot) {
            const int j = c++;
            if (j >= childEnd) {
                atomicOr(counters + kCntOverflow, 1);
                return;
            }
            nx.rO[j] = make_float4(v.g.P.x, v.g.P.y, v.g.P.z, bitsf(v.key));
            nx.rD[j] = make_float4(dir.x, dir.y, dir.z, bitsf(v.g.src));
            nx.tree[j] = v.tc * 4u + slot;
        };
        // the first child's direction was computed before allocation (firstChildDir)
        if (v.wantD) emit(v.dir0, 1u);
        if (v.wantS) emit(v.wantD ? reflect(v.d, v.g.N) : v.dir0, 2u);
        if (v.wantT) emit(v.wantD || v.wantS ? refract(v.d, v.g.N, 1.0F / v.ior) : v.dir0, 3u);
    }
    const int mask = (v.wantD ? 1 : 0) | (v.wantS ? 2 : 0) | (v.wantT ? 4 : 0);
    lv.vtx[i] = make_int4(v.mat, shadowBase, childBase, (v.nShadow << 3) | mask);
}

// direction of a vertex's first child: diffuse (PathTracer.cpp:90-91), else specular
// (:118-120), else transmission (:129-131)
__device__ __forceinline__ v3 firstChildDir(const ShadeState& v) {
    if (v.wantD) return cosineHemisphere(v.g.N, v.hcos, v.hsin, v.hemi2);
    if (v.wantS) return reflect(v.d, v.g.N);
    return refract(v.d, v.g.N, 1.0F / v.ior);
}

// kFull: the general kernel (textures, counting); the lean instantiation (no
// texture, compaction only, no statistics) needs fewer registers: 65 VGPRs instead of 103, so
// 7 waves per SIMD instead of 4, and reads the materials and lights (eight of a vertex's 64-B
// gathers, from tables of a few KB) from a copy in LDS instead of through the texture path,
// which the hit, ray and shading-record gathers keep busy.  (kShadeLdsTable: the launch falls
// back to the general kernel for scenes whose tables do not fit.)
constexpr int kShadeLdsTable = 256;  // float4: 4 per material, then 4 per light
// kRegen (level 1, tuning key 33 = 2): the camera rays regenerated here (cameraRay on ra, the
// function the packet walk generated them with: the same bits) instead of read from lv's records
template <int kShader, bool kFull, bool kRegen>
__global__ __launch_bounds__(kBlock) void k_shade(DScene s, Level lv, Level nx, int* counters, int level, ShadeArgs a,
                                                  int deadNext, RaygenArgs ra) {
    __shared__ float4 tab[kFull ? 1 : kShadeLdsTable];
    if constexpr (!kFull) {
        const int nm = 4 * s.nMats, nt = nm + 4 * s.nLights;
        for (int k = static_cast<int>(threadIdx.x); k < nt; k += kBlock) tab[k] = k < nm ? s.mats[k] : s.lights[k - nm];
        __syncthreads();
    }
    const float4* const mats = kFull ? s.mats : tab;
    const float4* const lights = kFull ? s.lights : tab + 4 * s.nMats;
    const SegMap map = segMap(counters, level, false, lv.segCap);
    const int count = map.total();
    static_assert(cntShadows(1, 1) == cntRays(2, 1) + 1, "pair layout");
    __shared__ unsigned long long allocLds[2 * (kBlock / 64 + 1)];
    const bool dead = deadNext != 0;
    int parity = 0;
    for (int base = static_cast<int>(blockIdx.x * blockDim.x); base < count;
         base += static_cast<int>(gridDim.x * blockDim.x)) {
        const int vi = base + static_cast<int>(threadIdx.x);
        const bool active = vi < count;
        const int i = active ? map.phys(vi) : 0;  // the vertex's slot
        ShadeState v{};
        if (active) {
            const float4 h = lv.hit[i];
            float4 kw = make_float4(0.0F, 0.0F, 0.0F, -1.0F);
            if (kFull && s.textured != 0) {  // also at the depth cap: rayTrace writes Kd before shade() returns
                kw = textureWrite(s, h);
                lv.kd[i] = kw;
                lv.last[i] = kw;
            }
            float4 o4, d4;
            uint32_t tc = 1u;
            if constexpr (kRegen) {
                cameraRay(ra, i, &o4, &d4);
            } else {
                o4 = lv.rO[i];
                d4 = lv.rD[i];
                tc = lv.tree[i];
            }
            v = shadePrepare<kShader>(s, o4, d4, h, tc, level, a, kw, mats, lights);
            if (!v.terminal && v.nChild > 0 && !dead) v.dir0 = firstChildDir(v);
        }
        // {rays of level+1, shadow rays of level}: one 64-bit allocation per block and iteration, in
        // the queue segment of this 256-vertex chunk (Queue segments, mrt_kernels.hpp: chunk c in
        // segment c % kQueueSegs, an even split whatever the grid; with a grid of a multiple of 8
        // workgroups, the segment of the workgroup's XCD)
        const int seg = static_cast<int>((static_cast<unsigned>(base) / blockDim.x) % kQueueSegs);
        auto* pair = reinterpret_cast<unsigned long long*>(counters + cntRays(level + 1, seg));
        const int childOff = seg * nx.segCap, shadowOff = seg * lv.shadowSegCap;
        int childBase, shadowBase;
        const int nC = active ? v.nChild : 0, nS = active ? v.nShadow : 0;
        blockAllocPair(pair, nC, nS, &childBase, &shadowBase, allocLds, parity);
        parity ^= 1;
        if (active)
            shadeEmit(s, v, i, lv, nx, shadowOff + shadowBase, childOff + childBase, shadowOff + lv.shadowSegCap,
                      childOff + nx.segCap, counters, a, dead, lights);
        if (kFull && a.stats != nullptr) {  // counting pass: shaded (non-terminal) vertices
            const uint64_t m = __ballot(active && !v.terminal);
            if (laneId() == 0 && m != 0) {
                atomicAdd(a.stats + kStatShaded, static_cast<unsigned long long>(__popcll(m)));
                atomicAdd(a.stats + kStatLevelShaded + level - 1, static_cast<unsigned long long>(__popcll(m)));
            }
        }
    }
}

// The same allocation for one wave (no barrier: the fused level-1 kernel's waves run their
// packets independently): one 64-bit atomic per wave and packet.
__device__ __forceinline__ void waveAllocPair(unsigned long long* pair, int nLo, int nHi, int* baseLo, int* baseHi) {
    const int lane = laneId();
    const unsigned long long v =
        (static_cast<unsigned long long>(static_cast<unsigned>(nHi)) << 32) | static_cast<unsigned>(nLo);
    unsigned long long x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    const unsigned long long total = __shfl(x, 63, 64);
    unsigned long long base = 0;
    if (lane == 0 && total != 0) base = atomicAdd(pair, total);
    base = __shfl(base, 0, 64);
    const unsigned long long e = base + (x - v);
    *baseLo = static_cast<int>(static_cast<unsigned>(e & 0xFFFFFFFFull));
    *baseHi = static_cast<int>(static_cast<unsigned>(e >> 32));
}

// Level 1 fused: the packet walk shades each packet's hits as soon as the packet is done
// (shadePrepare / shadeEmit of k_shade, the lean form), so the camera rays' shading runs inside
// the latency-bound packet walk instead of as a separate launch after it.  Same vertex records,
// shadow and child rays as k_shade (queue order differs, as it does between launches).
template <int kShader>
struct PacketShade {
    const DScene* s;
    Level lv, nx;
    int* counters;
    int level;
    ShadeArgs a;
    bool dead;
    __device__ __forceinline__ void operator()(int i, bool valid, float4 o4, float4 d4, float4 h) const {
        ShadeState v{};
        if (valid) {  // (tree code 1: a camera ray)
            v = shadePrepare<kShader>(*s, o4, d4, h, 1u, level, a, make_float4(0.0F, 0.0F, 0.0F, -1.0F), s->mats, s->lights);
            if (!v.terminal && v.nChild > 0 && !dead) v.dir0 = firstChildDir(v);
        }
        int childBase, shadowBase;
        // the packet's queue segment (Queue segments, mrt_kernels.hpp): its 64 paths' block
        const int seg = static_cast<int>((static_cast<unsigned>(__builtin_amdgcn_readfirstlane(i)) >> 6) % kQueueSegs);
        waveAllocPair(reinterpret_cast<unsigned long long*>(counters + cntRays(level + 1, seg)), valid ? v.nChild : 0,
                      valid ? v.nShadow : 0, &childBase, &shadowBase);
        const int childOff = seg * nx.segCap, shadowOff = seg * lv.shadowSegCap;
        if (valid)
            shadeEmit(*s, v, i, lv, nx, shadowOff + shadowBase, childOff + childBase, shadowOff + lv.shadowSegCap,
                      childOff + nx.segCap, counters, a, dead, s->lights);
    }
};

// ... and its camera rays are generated where they are walked (cameraRay, k_raygen's function):
// level 1's ray records are not written or read
struct PacketRays {
    const RaygenArgs* a;
    __device__ __forceinline__ void operator()(int i, float4* o4, float4* d4) const { cameraRay(*a, i, o4, d4); }
};

#ifndef MRT_FUSED_WAVES
#define MRT_FUSED_WAVES 6
#endif
template <int kShader, int kCull>
__global__ __launch_bounds__(kWalkThreads, MRT_FUSED_WAVES) void k_trace_packet_shade(DScene s, Level lv, Level nx, int* counters,
                                                                         int level, ShadeArgs a, int deadNext,
                                                                         int2* gstack, int gdepth, RaygenArgs ra) {
    __shared__ int2 ldsStack[kWalkStack * kWalkThreads];  // per-lane fallback walks only
    __shared__ int waveStacks[kWalkThreads / 64][kPacketStack];
    auto st = makeWalkStack<kCull>(ldsStack, gstack, gdepth);
    if (blockIdx.x == 0 && threadIdx.x == 0) denseCounts(counters, level, false, ra.nPaths, lv.segCap);  // (k_raygen's)
    const int count = min(ra.nPaths, lv.cap);
    int* fetch = counters + kCntFetchShards + level * kMaxFetchShards * kFetchStride;
    TravCount cnt{0u, 0u};
    const PacketShade<kShader> post{&s, lv, nx, counters, level, a, deadNext != 0};
    tracePacket<false, kCull>(s, lv.rO, lv.rD, lv.hit, count, fetch, st, &cnt, waveStacks[threadIdx.x / 64], post,
                              PacketRays{&ra});
}

// Single-level shaders: the camera ray's shade() spawns no rays, so the result is final here.
//   DepthMap (DepthMap.cpp:13-18), DiffuseMaterial (DiffuseMaterial.cpp:12-28),
//   NoShadows (NoShadows.cpp:13-44: direct light without shadow rays + ambient).
template <int kShader>
__global__ __launch_bounds__(kBlock) void k_shade_simple(DScene s, Level lv, int* counters, int level, ShadeArgs a) {
    const SegMap map = segMap(counters, level, false, lv.segCap);
    for (int vi = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); vi < map.total();
         vi += static_cast<int>(gridDim.x * blockDim.x)) {
        const int i = map.phys(vi);
        const float4 o4 = lv.rO[i];
        const float4 d4 = lv.rD[i];
        const float4 h = lv.hit[i];
        const uint32_t code = fbits(h.w);
        const uint32_t kind = primKind(code);
        v3 rgb{0.0F, 0.0F, 0.0F};
        float hitLight = 0.0F;
        if (kind != kMiss) {  // Shader.cpp:122: shade only on a hit
            v3 Le, Kd{0, 0, 0}, Ks{0, 0, 0}, Kt{0, 0, 0};
            {
                // a light hit carries the light's own material (Light::radiance_, AreaLight.cpp:32-41)
                const int mi = kind == kLight ? __float_as_int(s.lights[4 * primIndex(code) + 3].w) : hitMaterial(s, code);
                const float4* m = s.mats + 4 * mi;
                Le = xyz(m[0]);
                Kd = xyz(m[1]);
                Ks = xyz(m[2]);
                Kt = xyz(m[3]);
                if (s.textured != 0 && kind != kLight) {
                    const float4 kw = textureWrite(s, h);
                    if (kw.w >= 0.0F) Kd = xyz(kw);
                }
            }
            if (kShader == kShaderDepthMap) {
                const v3 mp{a.maxPoint[0], a.maxPoint[1], a.maxPoint[2]};
                const float maxDist = length(mp - xyz(o4)) * 1.1F;
                const float depth = stdmax((maxDist - h.x) / maxDist, 0.0F);
                rgb = v3{depth, depth, depth};
            } else if (kShader == kShaderDiffuse) {
                if (hasPositive(Kd)) {
                    rgb = Kd;
                } else if (hasPositive(Ks)) {
                    rgb = Ks;
                } else if (hasPositive(Kt)) {
                    rgb = Kt;
                } else if (hasPositive(Le)) {
                    rgb = Le;
                }
            } else if (hasPositive(Le)) {  // NoShadows
                rgb = Le;
                hitLight = 1.0F;
            } else {
                if (hasPositive(Kd) && s.nLights > 0) {
                    const uint32_t key = fbits(o4.w);
                    const uint32_t tc = lv.tree[i];
                    const HitGeom g = hitGeometry(s, xyz(o4), xyz(d4), h);
                    for (int k = 0; k < a.samplesLight; ++k) {
                        v3 ld, lc;
                        float dist;
                        if (lightSample(s, g, s.tables[sampleIndex(key, tc, purposeLightPick(k))].x,
                                        s.tables[sampleIndex(key, tc, purposeLightR(k))].y,
                                        s.tables[sampleIndex(key, tc, purposeLightS(k))].y, &ld, &dist, &lc, s.lights))
                            rgb = rgb + lc;  // Le * cosNl
                    }
                    rgb = rgb * Kd;
                    rgb = rgb / static_cast<float>(a.samplesLight);
                }
                rgb = rgb + Kd * 0.1F;
            }
        }
        lv.res[i] = make_float4(rgb.x, rgb.y, rgb.z, hitLight);
        lv.vtx[i] = make_int4(-1, 0, 0, 0);
    }
}

// ---------------------------------------------------------------------------------------
// kTex: a textured scene (the Kd replay below); untextured scenes run the lean instantiation
// Vertex i of level `level`: its radiance from its shadow rays' flags and its children's results,
// in the reference's float-op order (Whitted.cpp:36-92, PathTracer.cpp:22-142).
// Returns the radiance (w: the hit-a-light flag), or for a terminal vertex (va.x < 0) the record
// k_shade wrote; kLast: write the textured scenes' last-texel record for the level above.
template <int kShader, bool kTex, bool kLast>
__device__ __forceinline__ float4 resolveValue(const DScene& s, const Level& lv, const Level& nx, int i, int level,
                                               const ShadeArgs& a, int deadChildren, int4 va) {
    {
        if (va.x < 0) return lv.res[i];  // terminal: res written by k_shade
        // children (consecutive from va.z in the order diffuse, specular, transmission); an
        // index past the queue only occurs in an overflowed pass, which is redone
        int c = va.z;
        int4 vb = make_int4(-1, -1, -1, 0);
        if (va.w & 1) vb.x = c++;
        if (va.w & 2) vb.y = c++;
        if (va.w & 4) vb.z = c++;
        if (vb.x >= nx.cap) vb.x = -1;
        if (vb.y >= nx.cap) vb.y = -1;
        if (vb.z >= nx.cap) vb.z = -1;
        // children at the depth cap: radiance 0, no light hit.  Whitted adds Ks * 0 / Kt * 0 and
        // PathTracer Kd * 0 (finite materials) to sums that start at +0, which leaves them as
        // they are, so an absent child gives the same bits
        if (deadChildren != 0) vb = make_int4(-1, -1, -1, 0);
        const int nShadow = va.w >> 3;
        const float4* m = s.mats + 4 * va.x;
        v3 Kd = xyz(m[1]);
        const v3 Ks = xyz(m[2]), Kt = xyz(m[3]);
        // textured scenes: Kd as shade() reads it - this hit's texel until a child's subtree
        // writes the material again (exact while at most one material is textured: the subtree
        // records keep only its last write)
        float4 lD = make_float4(0.0F, 0.0F, 0.0F, -1.0F), lS = lD, lT = lD, own = lD;
        if (kTex) {
            own = lv.kd[i];
            if (own.w >= 0.0F) Kd = xyz(own);
            if (vb.x >= 0) lD = nx.last[vb.x];
            if (vb.y >= 0) lS = nx.last[vb.y];
            if (vb.z >= 0) lT = nx.last[vb.z];
        }
        const float matF = static_cast<float>(va.x);
        const bool direct = hasPositive(Kd) && s.nLights > 0;
        v3 Ld{0.0F, 0.0F, 0.0F};
        if (direct) {
            for (int k = 0; k < nShadow; ++k) {
                const int j = va.y + k;
                if (j >= lv.shadowCap) break;
                const float4 c = lv.sC[j];
                if (c.w == 0.0F) Ld = Ld + xyz(c);
            }
            Ld = Ld * Kd;
            Ld = Ld / static_cast<float>(a.samplesLight);
        }
        float4 out;
        if (kShader == kShaderWhitted) {  // Whitted.cpp:36-92
            v3 rgb = Ld;
            if (hasPositive(Ks) && vb.y >= 0) rgb = rgb + Ks * xyz(nx.res[vb.y]);
            if (hasPositive(Kt) && vb.z >= 0) rgb = rgb + Kt * xyz(nx.res[vb.z]);
            // the ambient term reads Kd after the specular and transmission subtrees
            const v3 KdAmb = lT.w == matF ? xyz(lT) : ((lT.w < 0.0F && lS.w == matF) ? xyz(lS) : Kd);
            rgb = rgb + KdAmb * 0.1F;
            out = make_float4(rgb.x, rgb.y, rgb.z, 0.0F);
        } else {  // PathTracer.cpp:127-142
            v3 LiD{0.0F, 0.0F, 0.0F}, LiS{0.0F, 0.0F, 0.0F}, LiT{0.0F, 0.0F, 0.0F};
            bool hitLight = false;
            if (vb.x >= 0) {
                const float4 r = nx.res[vb.x];
                hitLight = r.w != 0.0F;
                const v3 KdD = lD.w == matF ? xyz(lD) : Kd;  // Kd after the diffuse subtree
                LiD = LiD + KdD * xyz(r);
                if (level > kRayDepthMin) LiD = LiD / (0.5F * 0.5F);
                if (hasPositive(Ld) && hitLight) LiD = v3{0.0F, 0.0F, 0.0F};
            }
            if (hasPositive(Ks) && vb.y >= 0) LiS = LiS + Ks * xyz(nx.res[vb.y]);
            if (hasPositive(Kt) && vb.z >= 0) LiT = LiT + Kt * xyz(nx.res[vb.z]);
            v3 rgb{0.0F, 0.0F, 0.0F};
            rgb = rgb + Ld;
            rgb = rgb + LiD;
            rgb = rgb + LiS;
            rgb = rgb + LiT;
            out = make_float4(rgb.x, rgb.y, rgb.z, hitLight ? 1.0F : 0.0F);
        }
        if (kTex && kLast) lv.last[i] = lT.w >= 0.0F ? lT : (lS.w >= 0.0F ? lS : (lD.w >= 0.0F ? lD : own));
        return out;
    }
}

template <int kShader, bool kTex>
__device__ __forceinline__ void resolveVertex(const DScene& s, const Level& lv, const Level& nx, int i, int level,
                                              const ShadeArgs& a, int deadChildren) {
    const int4 va = lv.vtx[i];
    if (va.x < 0) return;  // terminal: res written by k_shade
    lv.res[i] = resolveValue<kShader, kTex, true>(s, lv, nx, i, level, a, deadChildren, va);
}

template <int kShader, bool kTex>
__global__ __launch_bounds__(256) void k_resolve(DScene s, Level lv, Level nx, int* counters, int level, ShadeArgs a,
                                                 int deadChildren) {
    const SegMap map = segMap(counters, level, false, lv.segCap);
    for (int vi = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); vi < map.total();
         vi += static_cast<int>(gridDim.x * blockDim.x))
        resolveVertex<kShader, kTex>(s, lv, nx, map.phys(vi), level, a, deadChildren);
}

// ---------------------------------------------------------------------------------------
// Pixel slot a.slotBase + q: incrementalAvg (Utils.cpp:66-90) of its samples, res[q * spp + s], in
// sample order, into the bitmap and / or the packed shard buffer.
__device__ __forceinline__ void accumulatePixel(const AccumArgs& a, const float4* res, int32_t* bitmap, int32_t* packed,
                                                int q) {
    const int slot = a.slotBase + q;
    int x, y;
    slotToXY(a.map, slot, &x, &y);
    const int idx = y * a.width + x;
    int32_t c = 0;  // the running average (progressive passes: sampleBase > 0)
    if (a.sampleBase > 0) c = bitmap != nullptr ? bitmap[idx] : (packed != nullptr ? packed[slot] : 0);
    for (int s = 0; s < a.spp; ++s) {
        const float4 r = res[q * a.spp + s];
        c = incrementalAvg(v3{r.x, r.y, r.z}, c, a.sampleBase + s + 1);
    }
    if (bitmap != nullptr) bitmap[idx] = c;
    if (packed != nullptr) packed[slot] = c;
}

__global__ __launch_bounds__(256) void k_accumulate(AccumArgs a, const float4* res, int32_t* bitmap, int32_t* packed) {
    const int q = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= a.nSlots) return;
    accumulatePixel(a, res, bitmap, packed, q);
}

// scatter a gathered, rank-packed buffer into the bitmap (multi-GPU frame assembly)
// every rank's shard in one launch: blockIdx.y = rank (of the batch)
__global__ __launch_bounds__(256) void k_unpack_ranks(UnpackArgs a, const int32_t* gathered, int32_t* bitmap) {
    const int k = static_cast<int>(blockIdx.y);
    const int q = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= a.n[k]) return;
    int x, y;
    slotToXY(a.maps[k], q, &x, &y);
    bitmap[y * a.width + x] = gathered[static_cast<size_t>(a.first + k) * static_cast<size_t>(a.stride) + q];
}

// primary-hit dump (config C2): per path slot (kind, index, t)
__global__ __launch_bounds__(256) void k_dump_hits(Level lv, int n, int32_t* kind, int32_t* index, float* t) {
    const int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const float4 h = lv.hit[i];
    const uint32_t code = fbits(h.w);
    kind[i] = static_cast<int32_t>(primKind(code));
    index[i] = primKind(code) == kMiss ? -1 : static_cast<int32_t>(primIndex(code));
    t[i] = h.x;
}

// One lane records the real-time counter (100 MHz) before and after a bounded spin of `ticks`: two
// launches on two streams overlap in time iff the streams feed different hardware queues.
__global__ void k_spin(unsigned long long* out, int slot, unsigned long long ticks) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long t = t0;
    for (int i = 0; i < (1 << 20) && t - t0 < ticks; ++i) {
        __builtin_amdgcn_s_sleep(8);
        t = __builtin_amdgcn_s_memrealtime();
    }
    out[2 * slot] = t0;
    out[2 * slot + 1] = t;
}

void launchSpin(unsigned long long* out, int slot, unsigned long long ticks, hipStream_t st) {
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st, out, slot, ticks);
}

// A chunk's ray counts into the pass statistics (thread 0), then (round 6) the statistics into the
// renderer's pinned host block (hostOut: read by the host after its stream synchronisation, instead
// of a device-to-host copy) and the device state reset for the next chunk or pass: the counters
// always, the statistics after the pass's last chunk (zeroStats) - so that no memset launch starts
// the next pass.
__global__ __launch_bounds__(256) void k_tally(int* counters, int maxLevel, unsigned long long* stats, int skippedLevel,
                                               unsigned long long* hostOut, int zeroStats) {
    if (threadIdx.x == 0) {
        unsigned long long rays = 0, shadows = 0;
        // a level's rays: the sum over its queue segments (the capped last level's are counted, never written)
        auto levelRays = [&](int l, bool sh) {
            unsigned long long n = 0;
            for (int g = 0; g < kQueueSegs; ++g)
                n += static_cast<unsigned long long>(counters[sh ? cntShadows(l, g) : cntRays(l, g)]);
            return n;
        };
        for (int l = 1; l <= maxLevel; ++l) {
            const unsigned long long r = levelRays(l, false), sh = levelRays(l, true);
            rays += r;
            shadows += sh;
            stats[kStatLevelRays + l - 1] += r;
            stats[kStatLevelShadows + l - 1] += sh;
        }
        stats[kStatRays] += rays;
        stats[kStatShadowRays] += shadows;
        stats[kStatPrimary] += levelRays(1, false);
        if (skippedLevel > 0) stats[kStatSkipped] += levelRays(skippedLevel, false);
        if (counters[kCntOverflow] != 0) stats[kStatOverflow] |= static_cast<unsigned long long>(counters[kCntOverflow]);
    }
    __syncthreads();
    if (hostOut != nullptr) {
        for (int k = static_cast<int>(threadIdx.x); k < kNumStats; k += static_cast<int>(blockDim.x)) {
            hostOut[k] = stats[k];
            if (zeroStats != 0) stats[k] = 0ull;
        }
        for (int k = static_cast<int>(threadIdx.x); k < kNumCounters; k += static_cast<int>(blockDim.x)) counters[k] = 0;
    }
}

// ---------------------------------------------------------------------------------------
// Device known-answer kernels: the SAME slab() / slabFinite() / triTest() the walks inline, on
// the reference's unit-test vectors (TestAABB.cpp:111-130, TestTriangle.cpp:347-433).
__global__ __launch_bounds__(64) void k_kat_slab(const float* boxes, const float* orig, const float* dir, int n,
                                                 int32_t* out) {
    const int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const float* b = boxes + 6 * i;
    const v3 o{orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]};
    const v3 d{dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]};
    const v3 inv{1.0F / d.x, 1.0F / d.y, 1.0F / d.z};
    float te;
    out[3 * i] = slab(b[0], b[1], b[2], b[3], b[4], b[5], o, inv, &te) ? 1 : 0;
    out[3 * i + 1] = slabFinite(b[0], b[1], b[2], b[3], b[4], b[5], o, inv, &te) ? 1 : 0;
    out[3 * i + 2] = finiteInv(inv) ? 1 : 0;  // slabFinite is used only for these rays
}

__global__ __launch_bounds__(64) void k_kat_triangle(const float* tris, const float* orig, const float* dir, int n,
                                                     int32_t* hit, float* tOut) {
    const int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const float* p = tris + 9 * i;  // A, B, C (Triangle.cpp:14-26: AB = B - A, AC = C - A)
    const float4 a4 = make_float4(p[0], p[1], p[2], 0.0F);
    const float4 ab4 = make_float4(p[3] - p[0], p[4] - p[1], p[5] - p[2], 0.0F);
    const float4 ac4 = make_float4(p[6] - p[0], p[7] - p[1], p[8] - p[2], 0.0F);
    const v3 o{orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]};
    const v3 d{dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]};
    float t = 0.0F, u, v;
    const bool h = triTest(a4, ab4, ac4, o, d, &t, &u, &v) && !(t < kEpsilon) && t < kRayLengthMax;
    hit[i] = h ? 1 : 0;
    tOut[i] = h ? t : 0.0F;
}

void launchKatSlab(const float* boxes, const float* orig, const float* dir, int n, int32_t* out, hipStream_t st) {
    hipLaunchKernelGGL(k_kat_slab, dim3((n + 63) / 64), dim3(64), 0, st, boxes, orig, dir, n, out);
}

void launchKatTriangle(const float* tris, const float* orig, const float* dir, int n, int32_t* hit, float* t,
                       hipStream_t st) {
    hipLaunchKernelGGL(k_kat_triangle, dim3((n + 63) / 64), dim3(64), 0, st, tris, orig, dir, n, hit, t);
}

// arbitrary rays into a level's queue (mrt_trace_rays): rO / rD or sO / sD / sC
__global__ __launch_bounds__(256) void k_load_rays(Level lv, const float* orig, const float* dir, const float* dist,
                                                   const uint32_t* src, int n, int any, int* counters) {
    const int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (i == 0) denseCounts(counters, 1, any != 0, n, any ? lv.shadowSegCap : lv.segCap);
    if (i >= n) return;
    const uint32_t code = src != nullptr ? src[i] : kNoPrim;
    if (any) {
        lv.sO[i] = make_float4(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2], bitsf(code));
        lv.sD[i] = make_float4(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2], dist[i]);
        lv.sC[i] = make_float4(0.0F, 0.0F, 0.0F, -1.0F);
    } else {
        lv.rO[i] = make_float4(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2], 0.0F);
        lv.rD[i] = make_float4(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2], bitsf(code));
        lv.tree[i] = 1u;
    }
}

void launchLoadRays(const Level& lv, const float* orig, const float* dir, const float* dist, const uint32_t* src, int n,
                    bool any, int* counters, hipStream_t st) {
    hipLaunchKernelGGL(k_load_rays, dim3(std::max(1, (n + 255) / 256)), dim3(256), 0, st, lv, orig, dir, dist, src, n,
                       any ? 1 : 0, counters);
}

// ---------------------------------------------------------------------------------------
// launch wrappers
void launchRaygen(const RaygenArgs& a, const Level& lv, int* counters, hipStream_t st) {
    const int blocks = (a.nPaths + 255) / 256;
    hipLaunchKernelGGL(k_raygen, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, a, lv, counters);
}

// Persistent grid: the kernel's own occupancy x CUs workgroups, capped by the thread count the
// spill stacks were sized for.
template <typename K>
int persistentGrid(K kernel, int slot, int maxThreads) {
    // Cached per device ordinal (a device group's shards launch from host threads of their own, each
    // with its own device current, and the GPUs of a group may differ in CU count): every thread
    // that fills an entry computes the same value for that device, so relaxed atomics suffice.
    constexpr int kDevices = 64;
    static std::atomic<int> occ[kDevices][24] = {};
    static std::atomic<int> cusCache[kDevices] = {};
    const int cap = std::max(1, maxThreads / kWalkThreads);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return cap;
    hipDeviceProp_t prop;
    if (dev < 0 || dev >= kDevices) {  // (beyond the cache: asked every time)
        int o = 0;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kernel, kWalkThreads, 0) != hipSuccess || o <= 0)
            return cap;
        return std::min(cap, o * prop.multiProcessorCount);
    }
    int cus = cusCache[dev].load(std::memory_order_relaxed);
    if (cus == 0) {
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return cap;
        cus = prop.multiProcessorCount;
        cusCache[dev].store(cus, std::memory_order_relaxed);
    }
    int o = occ[dev][slot].load(std::memory_order_relaxed);
    if (o == 0) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kernel, kWalkThreads, 0) != hipSuccess) o = 0;
        occ[dev][slot].store(o, std::memory_order_relaxed);
    }
    return o > 0 ? std::min(cap, o * cus) : cap;
}

// variant 0 (reference walk, never culls) and variant 1 in each cull mode; slot: occupancy cache
#define MRT_LAUNCH_ONE(KERNEL, V, C, SLOT)                                                                      \
    do {                                                                                                       \
        const int g = std::max(1, persistentGrid(KERNEL<false, V, C>, SLOT, maxThreads) * gridPct / 100);    \
        if (countStats)                                                                                        \
            hipLaunchKernelGGL((KERNEL<true, V, C>), dim3(g), dim3(kWalkThreads), 0, st, s, lv, counters, level, gstack, gdepth, stats); \
        else                                                                                                   \
            hipLaunchKernelGGL((KERNEL<false, V, C>), dim3(g), dim3(kWalkThreads), 0, st, s, lv, counters, level, gstack, gdepth, stats); \
    } while (0)
#define MRT_LAUNCH_WALK(KERNEL, SLOT)                                                                           \
    do {                                                                                                       \
        if (s.variant == 0) MRT_LAUNCH_ONE(KERNEL, 0, kCullNone, SLOT);                                        \
        else if (s.cull == kCullFast) MRT_LAUNCH_ONE(KERNEL, 1, kCullFast, SLOT + 1);                          \
        else if (s.cull == kCullCertified) MRT_LAUNCH_ONE(KERNEL, 1, kCullCertified, SLOT + 2);                \
        else if (s.cull == kCullExact) MRT_LAUNCH_ONE(KERNEL, 1, kCullExact, SLOT + 4);                        \
        else MRT_LAUNCH_ONE(KERNEL, 1, kCullNone, SLOT + 3);                                                   \
    } while (0)

bool packetLevel1(const DScene& s) {
    return s.accel == kAccBVH && s.packet != 0 && s.variant == 1 && (s.cull == kCullNone || s.cull == kCullExact);
}

void launchTrace(const DScene& s, const Level& lv, int* counters, int level, int2* gstack, int gdepth,
                 unsigned long long* stats, bool countStats, int maxThreads, hipStream_t st, const RaygenArgs* gen) {
    if (s.accel != kAccBVH) {
        hipLaunchKernelGGL((k_trace_other<false>), dim3(1024), dim3(256), 0, st, s, lv, counters, level);
        return;
    }
    const int gridPct = 100;
    if (level == 1 && packetLevel1(s)) {
        const int g = std::max(1, gen != nullptr ? persistentGrid(k_trace_packet<false, kCullExact, true>, 11, maxThreads)
                                                  : persistentGrid(k_trace_packet<false, kCullExact, false>, 10, maxThreads));
        const RaygenArgs ra = gen != nullptr ? *gen : RaygenArgs{};
#define MRT_LAUNCH_PACKET(CNT, C, GEN)                                                                        \
        hipLaunchKernelGGL((k_trace_packet<CNT, C, GEN>), dim3(g), dim3(kWalkThreads), 0, st, s, lv, counters, level, \
                           gstack, gdepth, stats, ra)
#define MRT_LAUNCH_PACKET_GEN(CNT, C)                     \
        do {                                              \
            if (gen != nullptr) MRT_LAUNCH_PACKET(CNT, C, true); \
            else MRT_LAUNCH_PACKET(CNT, C, false);        \
        } while (0)
        if (s.cull == kCullExact) {
            if (countStats) MRT_LAUNCH_PACKET_GEN(true, kCullExact);
            else MRT_LAUNCH_PACKET_GEN(false, kCullExact);
        } else {
            if (countStats) MRT_LAUNCH_PACKET_GEN(true, kCullNone);
            else MRT_LAUNCH_PACKET_GEN(false, kCullNone);
        }
#undef MRT_LAUNCH_PACKET_GEN
#undef MRT_LAUNCH_PACKET
        return;
    }
    MRT_LAUNCH_WALK(k_trace, 0);
}

void launchShadow(const DScene& s, const Level& lv, int* counters, int level, int2* gstack, int gdepth,
                  unsigned long long* stats, bool countStats, int maxThreads, hipStream_t st, int gridPct) {
    if (s.accel != kAccBVH) {
        hipLaunchKernelGGL((k_trace_other<true>), dim3(1024), dim3(256), 0, st, s, lv, counters, level);
        return;
    }
    MRT_LAUNCH_WALK(k_shadow, 5);
}

bool canFuseLevel1(int shader, const DScene& s, const ShadeArgs& a) {
    return s.fuseShade != 0 && s.accel == kAccBVH && s.packet != 0 && s.variant == 1 &&
           (s.cull == kCullNone || s.cull == kCullExact) && (shader == kShaderWhitted || shader == kShaderPathTracer) &&
           s.textured == 0 && a.stats == nullptr && s.leanShade != 0;
}

void launchTraceShadeFused(int shader, const DScene& s, const Level& lv, const Level& nx, int* counters, int level,
                           const ShadeArgs& a, int2* gstack, int gdepth, int maxThreads, hipStream_t st, bool deadNext,
                           const RaygenArgs& ra) {
    const int dead = deadNext ? 1 : 0;
#define MRT_LAUNCH_FUSED(SH, C)                                                                                  \
    do {                                                                                                         \
        const int g = std::max(1, persistentGrid(k_trace_packet_shade<SH, C>, 12 + (SH == kShaderWhitted ? 0 : 1) + \
                                                 (C == kCullExact ? 0 : 2), maxThreads));                         \
        hipLaunchKernelGGL((k_trace_packet_shade<SH, C>), dim3(g), dim3(kWalkThreads), 0, st, s, lv, nx, counters,  \
                           level, a, dead, gstack, gdepth, ra);                                                 \
    } while (0)
    if (shader == kShaderPathTracer) {
        if (s.cull == kCullExact) MRT_LAUNCH_FUSED(kShaderPathTracer, kCullExact);
        else MRT_LAUNCH_FUSED(kShaderPathTracer, kCullNone);
    } else {
        if (s.cull == kCullExact) MRT_LAUNCH_FUSED(kShaderWhitted, kCullExact);
        else MRT_LAUNCH_FUSED(kShaderWhitted, kCullNone);
    }
#undef MRT_LAUNCH_FUSED
}

void launchShade(int shader, const DScene& s, const Level& lv, const Level& nx, int* counters, int level,
                 const ShadeArgs& a, int grid, hipStream_t st, bool deadNext, const RaygenArgs* regen) {
    const int dead = deadNext ? 1 : 0;
    const RaygenArgs ra = regen != nullptr ? *regen : RaygenArgs{};
    // (a separate instantiation: the regeneration in the shared one cost 8 VGPRs and a wave per SIMD)
#define MRT_LAUNCH_SHADE_ONE(SH, FULL, RG)                                                                 \
    hipLaunchKernelGGL((k_shade<SH, FULL, RG>), dim3(grid), dim3(kBlock), 0, st, s, lv, nx, counters, level, a, \
                       dead, ra)
#define MRT_LAUNCH_SHADE(SH, FULL)                         \
    do {                                                   \
        if (regen != nullptr) MRT_LAUNCH_SHADE_ONE(SH, FULL, true); \
        else MRT_LAUNCH_SHADE_ONE(SH, FULL, false);        \
    } while (0)
    const bool full = s.textured != 0 || a.stats != nullptr || s.leanShade == 0 ||
                      4 * (s.nMats + s.nLights) > kShadeLdsTable;
    switch (shader) {
        case kShaderWhitted:
            if (full)
                MRT_LAUNCH_SHADE(kShaderWhitted, true);
            else
                MRT_LAUNCH_SHADE(kShaderWhitted, false);
            break;
        case kShaderPathTracer:
            if (full)
                MRT_LAUNCH_SHADE(kShaderPathTracer, true);
            else
                MRT_LAUNCH_SHADE(kShaderPathTracer, false);
            break;
        case kShaderDepthMap:
            hipLaunchKernelGGL(k_shade_simple<kShaderDepthMap>, dim3(grid), dim3(kBlock), 0, st, s, lv, counters, level, a);
            break;
        case kShaderDiffuse:
            hipLaunchKernelGGL(k_shade_simple<kShaderDiffuse>, dim3(grid), dim3(kBlock), 0, st, s, lv, counters, level, a);
            break;
        default:
            hipLaunchKernelGGL(k_shade_simple<kShaderNoShadows>, dim3(grid), dim3(kBlock), 0, st, s, lv, counters, level, a);
            break;
    }
#undef MRT_LAUNCH_SHADE
#undef MRT_LAUNCH_SHADE_ONE
}

void launchResolve(int shader, const DScene& s, const Level& lv, const Level& nx, int* counters, int level,
                   const ShadeArgs& a, int grid, hipStream_t st, bool deadChildren) {
    const int dead = deadChildren ? 1 : 0;
    const bool tex = s.textured != 0;
    if (shader == kShaderPathTracer) {
        if (tex)
            hipLaunchKernelGGL((k_resolve<kShaderPathTracer, true>), dim3(grid), dim3(256), 0, st, s, lv, nx, counters, level, a, dead);
        else
            hipLaunchKernelGGL((k_resolve<kShaderPathTracer, false>), dim3(grid), dim3(256), 0, st, s, lv, nx, counters, level, a, dead);
    } else if (shader == kShaderWhitted) {
        if (tex)
            hipLaunchKernelGGL((k_resolve<kShaderWhitted, true>), dim3(grid), dim3(256), 0, st, s, lv, nx, counters, level, a, dead);
        else
            hipLaunchKernelGGL((k_resolve<kShaderWhitted, false>), dim3(grid), dim3(256), 0, st, s, lv, nx, counters, level, a, dead);
    }  // single-level shaders: k_shade_simple wrote the final results
}

// Level 1's resolve and the accumulation in one launch (round 6, tuning key 34): a thread per path
// (q * spp + s, level 1) resolves its camera-ray vertex as k_resolve does, and the first lane of each
// pixel slot's spp consecutive lanes (spp divides 64, so a slot's samples share a wave) pulls the
// others' radiance and averages them in sample order as k_accumulate does, so level 1's radiance
// records are never written or re-read.  The same resolveValue and incrementalAvg on the same
// inputs: the same bits.  (A thread per slot resolving its samples one after another measured
// slower, C4 13.65 -> 13.78 ms: four dependent gather chains per thread.)
template <int kShader, bool kTex>
__global__ __launch_bounds__(256) void k_resolve_accumulate(DScene s, Level lv, Level nx, ShadeArgs sa, int deadChildren,
                                                            AccumArgs a, int32_t* bitmap, int32_t* packed) {
    const int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    const int n = a.nSlots * a.spp;
    float4 r = make_float4(0.0F, 0.0F, 0.0F, 0.0F);
    if (i < n) r = resolveValue<kShader, kTex, false>(s, lv, nx, i, 1, sa, deadChildren, lv.vtx[i]);
    const int k = i % a.spp;  // this path's sample; lanes i - k .. i - k + spp - 1 hold its slot's
    int32_t c = 0;
    for (int j = 0; j < a.spp; ++j) {  // (wave-uniform trip count)
        const int from = static_cast<int>(threadIdx.x & 63u) + j;  // lane of sample j when k == 0
        const float x = __shfl(r.x, from, 64), y = __shfl(r.y, from, 64), z = __shfl(r.z, from, 64);
        if (k == 0 && i < n) {
            if (j == 0 && a.sampleBase > 0) {  // the running average (progressive passes)
                const int slot = a.slotBase + i / a.spp;
                int px, py;
                slotToXY(a.map, slot, &px, &py);
                c = bitmap != nullptr ? bitmap[py * a.width + px] : (packed != nullptr ? packed[slot] : 0);
            }
            c = incrementalAvg(v3{x, y, z}, c, a.sampleBase + j + 1);
        }
    }
    if (k == 0 && i < n) {
        const int slot = a.slotBase + i / a.spp;
        int px, py;
        slotToXY(a.map, slot, &px, &py);
        if (bitmap != nullptr) bitmap[py * a.width + px] = c;
        if (packed != nullptr) packed[slot] = c;
    }
}

bool launchResolveAccumulate(int shader, const DScene& s, const Level& lv, const Level& nx, const ShadeArgs& sa,
                             bool deadChildren, const AccumArgs& a, int32_t* bitmap, int32_t* packed, hipStream_t st) {
    if (a.spp <= 0 || 64 % a.spp != 0) return false;  // a slot's samples must share a wave
    const int dead = deadChildren ? 1 : 0;
    const int blocks = std::max(1, (a.nSlots * a.spp + 255) / 256);
#define MRT_LAUNCH_RA(SH, TEX)                                                                                  \
    hipLaunchKernelGGL((k_resolve_accumulate<SH, TEX>), dim3(blocks), dim3(256), 0, st, s, lv, nx, sa, dead, a, \
                       bitmap, packed)
    const bool tex = s.textured != 0;
    if (shader == kShaderPathTracer) {
        if (tex) MRT_LAUNCH_RA(kShaderPathTracer, true);
        else MRT_LAUNCH_RA(kShaderPathTracer, false);
    } else if (shader == kShaderWhitted) {
        if (tex) MRT_LAUNCH_RA(kShaderWhitted, true);
        else MRT_LAUNCH_RA(kShaderWhitted, false);
    } else {
        return false;
    }
#undef MRT_LAUNCH_RA
    return true;
}

void launchAccumulate(const AccumArgs& a, const float4* res, int32_t* bitmap, int32_t* packed, hipStream_t st) {
    const int blocks = (a.nSlots + 255) / 256;
    hipLaunchKernelGGL(k_accumulate, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, a, res, bitmap, packed);
}

void launchUnpackRanks(const UnpackArgs& a, int ranks, int maxN, const int32_t* gathered, int32_t* bitmap,
                       hipStream_t st) {
    const int blocks = (maxN + 255) / 256;
    if (ranks <= 0 || blocks <= 0) return;
    hipLaunchKernelGGL(k_unpack_ranks, dim3(blocks, ranks), dim3(256), 0, st, a, gathered, bitmap);
}

void launchDumpHits(const Level& lv, int n, int32_t* kind, int32_t* index, float* t, hipStream_t st) {
    const int blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_dump_hits, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, lv, n, kind, index, t);
}

void launchTally(int* counters, int maxLevel, unsigned long long* stats, hipStream_t st, int skippedLevel,
                 unsigned long long* hostOut, bool zeroStats) {
    hipLaunchKernelGGL(k_tally, dim3(1), dim3(256), 0, st, counters, maxLevel, stats, skippedLevel, hostOut,
                       zeroStats ? 1 : 0);
}

int traceResidentThreadsPerCU() {
    // the spill stacks are sized for the walk with the most resident threads
    int best = kWalkThreads;
    const void* kernels[] = {reinterpret_cast<const void*>(k_trace<false, 0, kCullNone>),
                             reinterpret_cast<const void*>(k_trace<false, 1, kCullFast>),
                             reinterpret_cast<const void*>(k_trace<false, 1, kCullCertified>),
                             reinterpret_cast<const void*>(k_trace<false, 1, kCullNone>),
                             reinterpret_cast<const void*>(k_trace<false, 1, kCullExact>),
                             reinterpret_cast<const void*>(k_shadow<false, 0, kCullNone>),
                             reinterpret_cast<const void*>(k_shadow<false, 1, kCullFast>),
                             reinterpret_cast<const void*>(k_shadow<false, 1, kCullCertified>),
                             reinterpret_cast<const void*>(k_shadow<false, 1, kCullNone>),
                             reinterpret_cast<const void*>(k_shadow<false, 1, kCullExact>),
                             reinterpret_cast<const void*>(k_trace_packet<false, kCullExact, false>),
                             reinterpret_cast<const void*>(k_trace_packet<false, kCullNone, false>)};
    for (const void* k : kernels) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, kWalkThreads, 0) == hipSuccess)
            best = std::max(best, n * kWalkThreads);
    }
    return best;
}

}  // namespace mrt
