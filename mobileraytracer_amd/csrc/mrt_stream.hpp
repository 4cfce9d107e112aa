// mrt_stream.hpp - one persistent launch for every level of a pass ("streaming" mode).
//
// The level-by-level wavefront (trace L -> shade L -> trace L+1 ...) waits at every level for
// its slowest ray: up to ~8x the mean walk, long enough that at small per-GPU frames (strong
// scaling) the texture path idles a third of the time.  Here one persistent kernel takes work
// from every level's queue as it appears: a lane whose closest-hit walk ends shades the vertex
// at once (shadePrepare / shadeEmit, the same code as k_shade) and publishes its children and
// shadow rays; any wave may pick them up in the same launch.  Results do not depend on the
// order in which rays are processed, so images are identical to the level-by-level path.
//
// Hand-off (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md "inter-workgroup
// visibility"): a producer reserves slots with an agent-scope atomic, stores the payload with
// `sc1` buffer stores, waits for its stores (`s_waitcnt vmcnt(0)`), then stores the slot's
// ready flag (`sc1`).  A consumer claims only reserved slots (compare-and-swap of the claim
// cursor against the allocation count), polls the slot's flag with `sc1` loads and reads the
// payload with `sc1` loads.  A producer never waits between reserving and flagging, so every
// poll ends; polls and the main loop are bounded anyway (error flag, never a hang).
// Termination: `pending` counts items (rays, shadow rays) that exist and are not finished; a
// shaded ray adds its children before it removes itself, so pending reaches 0 only at the end.
#pragma once

#include "mrt_kernels.hpp"
#include "mrt_trace_ww.hpp"

namespace mrt {

constexpr int kStreamMaxPolls = 1 << 22;    // per claimed slot
constexpr int kStreamMaxIdle = 1 << 22;     // idle iterations of one wave (no item anywhere)
constexpr int kStreamErrPoll = 1;
constexpr int kStreamErrIdle = 2;

struct StreamArgs {
    Level lv[kMaxLevels];  // levels 1..nLevels (+ nLevels + 1: no rays)
    int nLevels;
    uint32_t epoch;        // ready flags equal to this are set in the current pass
    ShadeArgs sa;
};

__device__ __forceinline__ int* streamCnt(int* counters, int level, int which) {  // which: 0..3
    return counters + kCntStream + (level * 4 + which) * kFetchStride;
}

__device__ __forceinline__ float4 sc1Load4(const float4* base, int j) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                          __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(base), static_cast<short>(0),
                                                                            0x7FFFFFFF, 0x00020000),
                                          static_cast<uint32_t>(j) * 16u, 0, 16));
}
__device__ __forceinline__ uint32_t sc1Load1(const uint32_t* base, int j) {
    return __builtin_amdgcn_raw_buffer_load_b32(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(base), static_cast<short>(0), 0x7FFFFFFF, 0x00020000),
        static_cast<uint32_t>(j) * 4u, 0, 16);
}

template <int kShader, int kWide, int kRefill, int kTop, bool kFastSlab>
__device__ __forceinline__ void streamLoop(const DScene& s, const StreamArgs& A, int* counters, TStack& st,
                                           const GNode* ldsTop) {
    const int lane = static_cast<int>(threadIdx.x & 63u);
    const int top = kTop > 0 ? min(kTop, s.triTop) : 0;
    const BufRes nodeBuf = bufferOf(s.triNodes);
    const BufRes triBuf = bufferOf(s.triGeom);
    int* pending = counters + kCntStream + kMaxLevels * 4 * kFetchStride;
    int* errorFlag = pending + kFetchStride;

    int item = -1, lvl = 0;
    bool any = false;  // shadow ray (any hit, tmax = bt)
    v3 o{0, 0, 0}, d{0, 0, 0}, inv{0, 0, 0};
    uint32_t src = 0, key = 0, tc = 0;
    float bt = kRayLengthMax;
    uint32_t bcode = kNoPrim;
    int ref = kRefDone;
    int leaf = 0;
    int idle = 0;
    int carry = 0;         // shadow rays found occluded since the last flush of `pending`
    bool waiting = false;  // item claimed, payload not loaded yet
    int qHint = 0;         // the queue this wave last took work from (wave-uniform)
    while (true) {
        // Lanes whose walk ended wait, like empty lanes, until kRefill of them are idle (or no
        // lane walks): shading then runs with most of the wave, not lane by lane.
        const bool fin = item >= 0 && !waiting && ref == kRefDone && leaf >= 0;
        const bool walking = item >= 0 && !waiting && !fin;
        const uint64_t walkMask = __ballot(walking);
        const bool batch = walkMask == 0 || __popcll(__ballot(!walking && !waiting)) >= kRefill;
        if (batch) {
            int delta = carry;  // this lane's change of `pending`
            carry = 0;
            // ---- walks that ended: shadow rays record occlusion, camera/bounce rays are shaded ----
            const bool shadeNow = fin && !any;
            if (fin && any) {
                A.lv[lvl].sC[item].w = 0.0F;  // unoccluded (occlusion was recorded in the leaf loop)
                delta -= 1;
                item = -1;
            }
            ShadeState v{};
            if (shadeNow) {
                for (int j = 0; j < s.nLights; ++j) {  // Shader.cpp:166-171
                    const float4* l = s.lights + 4 * j;
                    const float4 a4 = l[0];
                    if (__float_as_int(a4.w) != 1) continue;
                    float t, u, w;
                    if (!triTest(a4, l[1], l[2], o, d, &t, &u, &w)) continue;
                    if (t < kEpsilon) continue;
                    const uint32_t code = encodePrim(kLight, static_cast<uint32_t>(j));
                    if (betterThan(t, code, bt, bcode)) {
                        bt = t;
                        bcode = code;
                    }
                }
                float u = 0.0F, w = 0.0F, t;
                const uint32_t kind = primKind(bcode);
                if (kind == kTriangle || kind == kLight) {
                    const float4* g = kind == kTriangle ? s.triGeom + 3 * primIndex(bcode) : s.lights + 4 * primIndex(bcode);
                    (void)triTest(g[0], g[1], g[2], o, d, &t, &u, &w);
                }
                v = shadePrepare<kShader>(s, make_float4(o.x, o.y, o.z, bitsf(key)), make_float4(d.x, d.y, d.z, 0.0F),
                                          make_float4(bt, u, w, bitsf(bcode)), tc, lvl, A.sa);
            }
            // allocation and emission, one level at a time (lanes may hold different levels)
            uint64_t todo = __ballot(shadeNow);
            int childBase = 0, shadowBase = 0, nChildOk = 0, nShadowOk = 0;
            while (todo != 0) {
                const int leader0 = __ffsll(static_cast<unsigned long long>(todo)) - 1;
                const int L = __builtin_amdgcn_readfirstlane(__shfl(lvl, leader0, 64));  // wave-uniform
                const bool mine = shadeNow && lvl == L;
                const uint64_t m = __ballot(mine);
                int nc = mine ? v.nChild : 0, ns = mine ? v.nShadow : 0;
    #pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int yc = __shfl_up(nc, off, 64), ys = __shfl_up(ns, off, 64);
                    if (lane >= off) {
                        nc += yc;
                        ns += ys;
                    }
                }
                const int totC = __shfl(nc, 63, 64), totS = __shfl(ns, 63, 64);
                int cb = 0, sb = 0;
                if (lane == leader0) {
                    if (totC > 0) cb = atomicAdd(streamCnt(counters, L + 1, 0), totC);
                    if (totS > 0) sb = atomicAdd(streamCnt(counters, L, 2), totS);
                }
                cb = __shfl(cb, leader0, 64);
                sb = __shfl(sb, leader0, 64);
                if (mine) {
                    childBase = cb + nc - v.nChild;
                    shadowBase = sb + ns - v.nShadow;
                    shadeEmit<true>(s, v, item, A.lv[L], A.lv[L + 1], shadowBase, childBase, counters, A.sa);
                    nChildOk = v.terminal ? 0 : max(0, min(v.nChild, A.lv[L + 1].cap - childBase));
                    nShadowOk = v.terminal ? 0 : max(0, min(v.nShadow, A.lv[L].shadowCap - shadowBase));
                }
                todo &= ~m;
            }
            if (__ballot(shadeNow) != 0) {
                // every payload store of this wave has landed before any of its flags
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (shadeNow) {
                    for (int k = 0; k < nChildOk; ++k)
                        __hip_atomic_store(A.lv[lvl + 1].ready + childBase + k, A.epoch, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    for (int k = 0; k < nShadowOk; ++k)
                        __hip_atomic_store(A.lv[lvl].sReady + shadowBase + k, A.epoch, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    delta += nChildOk + nShadowOk - 1;
                    item = -1;
                }
            }
            // ---- pending: one atomic per wave and iteration ----
            {
                int sum = delta;
                for (int off = 32; off > 0; off >>= 1) sum += __shfl_down(sum, off, 64);
                if (lane == 0 && sum != 0) atomicAdd(pending, sum);
            }
            // ---- refill: idle lanes claim slots (one atomic per wave and queue); a claimed slot
            // may still be empty (its producer has not reserved or flagged it yet): the lane then
            // waits without holding up the wave, and gives the slot up once nothing is pending ----
            const uint64_t needMask = __ballot(item < 0);
            if (needMask != 0) {
                uint64_t open = needMask;
                const int nq = 2 * A.nLevels - 1;  // rays of 1..n, shadow rays of 1..n-1
                for (int k = 0; k < nq && open != 0; ++k) {
                    const int q = (qHint + k) % nq;
                    const int L = q < A.nLevels ? q + 1 : q - A.nLevels + 1;
                    const bool isShadow = q >= A.nLevels;
                    const int cap = isShadow ? A.lv[L].shadowCap : A.lv[L].cap;
                    int* allocC = L == 1 && !isShadow ? counters + cntRays(1) : streamCnt(counters, L, isShadow ? 2 : 0);
                    int* claimC = streamCnt(counters, L, isShadow ? 3 : 1);
                    const int leader = __ffsll(static_cast<unsigned long long>(open)) - 1;
                    int base = 0, n = 0;
                    if (lane == leader) {
                        const int c = __hip_atomic_load(claimC, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const int al = min(__hip_atomic_load(allocC, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), cap);
                        if (c < al) {
                            n = min(__popcll(open), al - c);
                            base = atomicAdd(claimC, n);  // racing waves may overshoot the allocation
                        }
                    }
                    base = __shfl(base, leader, 64);
                    n = __shfl(n, leader, 64);
                    if (n > 0) {
                        qHint = q;
                        const bool mine = ((open >> lane) & 1ull) != 0;
                        const int rank = lanesBelowIn(open);
                        if (mine && rank < n) {
                            item = base + rank;
                            lvl = L;
                            any = isShadow;
                            waiting = true;
                        }
                        open = __ballot(mine && rank >= n);
                    }
                }
            }
        }  // batch
        // ---- claimed slots whose payload is ready become active ----
        if (waiting) {
            const Level& Lv = A.lv[lvl];
            const int cap = any ? Lv.shadowCap : Lv.cap;
            bool ready = false;
            if (item >= cap) {
                ready = false;
            } else if (!any && lvl == 1) {
                ready = item < counters[cntRays(1)];
            } else {
                ready = __hip_atomic_load((any ? Lv.sReady : Lv.ready) + item, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                        A.epoch;
            }
            if (ready) {
                waiting = false;
                float4 o4, d4;
                if (any) {
                    o4 = sc1Load4(Lv.sO, item);
                    d4 = sc1Load4(Lv.sD, item);
                } else if (lvl > 1) {
                    o4 = sc1Load4(Lv.rO, item);
                    d4 = sc1Load4(Lv.rD, item);
                    tc = sc1Load1(Lv.tree, item);
                } else {
                    o4 = Lv.rO[item];
                    d4 = Lv.rD[item];
                    tc = Lv.tree[item];
                }
                o = xyz(o4);
                d = xyz(d4);
                inv = v3{1.0F / d.x, 1.0F / d.y, 1.0F / d.z};
                ref = kRefDone;
                leaf = 0;
                st.sp = 0;
                Best b;
                bool occluded = false;
                TravCount none{0u, 0u};
                if (any) {
                    src = fbits(o4.w);
                    b = Best{d4.w, 0.0F, 0.0F, kNoPrim};
                    occluded = traverse<kPlane, true>(s, s.planeNodes, s.planeRoot, o, d, inv, src, &b, st, &none) ||
                               traverse<kSphere, true>(s, s.sphereNodes, s.sphereRoot, o, d, inv, src, &b, st, &none);
                } else {
                    key = fbits(o4.w);
                    src = fbits(d4.w);
                    b = Best{kRayLengthMax, 0.0F, 0.0F, kNoPrim};
                    traverse<kPlane, false>(s, s.planeNodes, s.planeRoot, o, d, inv, src, &b, st, &none);
                    traverse<kSphere, false>(s, s.sphereNodes, s.sphereRoot, o, d, inv, src, &b, st, &none);
                }
                bt = b.t;
                bcode = b.code;
                if (occluded) {
                    Lv.sC[item].w = 1.0F;
                    item = -1;
                    carry -= 1;
                } else {
                    float te;
                    const GRoot& r = s.triRoot;
                    if (r.count > 0 && slab(r.bmin[0], r.bmin[1], r.bmin[2], r.bmax[0], r.bmax[1], r.bmax[2], o, inv, &te)) {
                        ref = r.ref;
                        if (ref < 0) {
                            leaf = ref;
                            ref = kRefDone;
                        }
                    }
                }
            }
        }
        const bool activeLane = item >= 0 && !waiting;
        if (__ballot(activeLane) == 0) {
            // nothing to walk: finished, or work still being produced by other waves
            int p = 0;
            if (lane == 0) p = __hip_atomic_load(pending, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            p = __shfl(p, 0, 64);
            if (p <= 0 && carry == 0) {
                if (__ballot(carry != 0) == 0) break;  // claimed-but-empty slots are given up
            }
            if (++idle > kStreamMaxIdle) {
                if (lane == 0) atomicOr(errorFlag, kStreamErrIdle);
                break;
            }
            if (idle < 64) {
                __builtin_amdgcn_s_sleep(1);
            } else {
                __builtin_amdgcn_s_sleep(8);
            }
            continue;
        }
        idle = 0;
        // ---- inner nodes until every active lane holds a postponed leaf ----
        while (static_cast<unsigned>(ref) < static_cast<unsigned>(kRefDone)) {
            const float curLim = bt + bt * kCullMargin;
            const bool finite = kFastSlab && __ballot(!finiteInv(inv)) == 0;
            TravCount none{0u, 0u};
            ref = innerStep2<kTop>(nodeBuf, ldsTop, top, ref, o, inv, curLim, s.cull != 0, st, &none, false, finite);
            if (ref < 0 && leaf >= 0) {
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
                const uint32_t off = static_cast<uint32_t>(j) * 48u;
                float t, u, w;
                if (!triTest(bload3(triBuf, off), bload3(triBuf, off + 16u), bload3(triBuf, off + 32u), o, d, &t, &u, &w))
                    continue;
                if (t < kEpsilon) continue;
                if (any) {
                    if (!(t >= bt)) {
                        hit = true;
                        break;
                    }
                } else if (betterThan(t, code, bt, bcode)) {
                    bt = t;
                    bcode = code;
                }
            }
            if (any && hit) {  // occluded: done
                A.lv[lvl].sC[item].w = 1.0F;
                carry -= 1;
                item = -1;
                st.sp = 0;
                ref = kRefDone;
                leaf = 0;
                break;
            }
            leaf = 0;
            if (ref < 0) {
                leaf = ref;
                ref = popCulled(st, bt + bt * kCullMargin, s.cull != 0);
            }
        }
    }
}

}  // namespace mrt
