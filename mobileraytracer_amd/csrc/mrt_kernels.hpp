// mrt_kernels.hpp - queue layouts, kernel argument blocks and launch wrappers.
#pragma once

#include "mrt_device.hpp"

namespace mrt {

constexpr int kShaderWhitted = 1;     // C_wrapper.cpp:155-160
constexpr int kShaderPathTracer = 2;  // C_wrapper.cpp:162-172
constexpr int kShaderDepthMap = 3;    // C_wrapper.cpp:175-179
constexpr int kShaderDiffuse = 4;     // C_wrapper.cpp:181-186 (DiffuseMaterial)
constexpr int kShaderNoShadows = 5;   // C_wrapper.cpp:188-193 (the switch's default: 0, 5, ...)
constexpr int kMaxLevels = 16;           // max ray depth + 2
constexpr int kTraceVariants = 2;        // 0: per-wave reference walk, 1: persistent while-while walk
constexpr int kDefaultTraceVariant = 1;
constexpr int kAccNaive = 1;  // Shader::Accelerator (Shader.hpp:20-24)
constexpr int kAccGrid = 2;
constexpr int kAccBVH = 3;
constexpr int kTopNodesMax = 64 * 4 / kWalkWidth;  // walk-tree nodes numbered breadth-first (4 KB staged in LDS by the walk)

// Queue segments (round 6).  Every queue a level's shading fills - the next level's rays, this level's
// shadow rays - is kQueueSegs segments of segCap / shadowSegCap slots (Level), each with its own
// counter pair on its own 256-B line: workgroup b allocates in segment b % kQueueSegs.  One counter
// for the whole queue made every allocation a same-address atomic, which queue at the memory side
// (a second such atomic per allocation cost +8.1 ms per C4 frame, spread over 8 lines +0.03 ms:
// profiles/r06_alloc_atomic_probe.txt).  A segment's rays are [g * segCap, g * segCap + count_g);
// consumers walk the segments (LevelQueue's cursors) or map a dense index over them (SegMap).
// Level 1 is one dense range [0, n) cut into segments of segCap (denseCounts).
#ifndef MRT_QUEUE_SEGS
#define MRT_QUEUE_SEGS 8
#endif
constexpr int kQueueSegs = MRT_QUEUE_SEGS;
// Device counters (ints).  Segment g's pair l = {rays of level l+1, shadow rays of level l} sits on
// two adjacent ints so k_shade allocates both with one 64-bit atomic per workgroup iteration.
constexpr int kCntSegStride = 64;                     // ints between segments' pair tables (>= 2 * (kMaxLevels + 1))
constexpr int kCntPairs = 0;                          // kQueueSegs tables
constexpr int kCntOverflow = kQueueSegs * kCntSegStride;
constexpr int kPacketStack = 128;  // the packet walk's wave-uniform stack entries (mrt_trace_packet.hpp)
#ifndef MRT_WALK_CURSORS
#define MRT_WALK_CURSORS 8
#endif
constexpr int kMaxFetchShards = MRT_WALK_CURSORS;     // work cursors per level (a multiple of the 8 XCD groups)
constexpr int kFetchStride = 32;                      // ints between cursors (a 128-byte line each)
constexpr int kCntFetchShards = kCntOverflow + kFetchStride;  // 2 kinds x kMaxLevels x kMaxFetchShards lines
constexpr int kNumCounters = kCntFetchShards + 2 * kMaxLevels * kMaxFetchShards * kFetchStride;
MRT_HD constexpr int cntRays(int level, int seg = 0) { return kCntPairs + seg * kCntSegStride + 2 * (level - 1); }
MRT_HD constexpr int cntShadows(int level, int seg = 0) { return kCntPairs + seg * kCntSegStride + 2 * level + 1; }
static_assert(kQueueSegs >= 1 && kQueueSegs <= kMaxFetchShards, "queue segments: one work cursor each at most");
static_assert(cntShadows(kMaxLevels) < kCntSegStride, "a segment's pairs within its line");

// 64-bit statistics accumulated on the device across a frame
constexpr int kStatRays = 0;        // rays of every level (camera + diffuse + specular + transmission)
constexpr int kStatShadowRays = 1;  // shadow rays
constexpr int kStatPrimary = 2;
constexpr int kStatNodes = 3;       // closest-hit kernel: child node records fetched (counting pass only)
constexpr int kStatTris = 4;        // closest-hit kernel: triangle tests (counting pass only)
constexpr int kStatOverflow = 5;
constexpr int kStatNodesShadow = 6; // any-hit kernel: child node records fetched (counting pass only)
constexpr int kStatTrisShadow = 7;  // any-hit kernel: triangle tests (counting pass only)
constexpr int kStatLevelRays = 8;                     // + level - 1: rays of each level
constexpr int kStatLevelShadows = 8 + kMaxLevels;     // + level - 1: shadow rays of each level
constexpr int kStatMaxNodesRay = 8 + 2 * kMaxLevels;  // counting builds: most node records of one ray
constexpr int kStatSkipped = kStatMaxNodesRay + 1;   // rays of a last level whose walk was skipped
constexpr int kStatShaded = kStatSkipped + 1;        // counting pass: vertices k_shade shaded (hit, not emissive, not capped)
constexpr int kStatShadeLaunches = kStatShaded + 1;  // k_shade launches of the frame
constexpr int kStatLeaves = kStatShadeLaunches + 1;  // counting pass: leaf records fetched, closest hit
constexpr int kStatLeavesShadow = kStatLeaves + 1;   // ... and any hit
// counting pass, closest hit, per level (+ level - 1): child records, triangle tests, leaf records
constexpr int kStatLevelNodes = kStatLeavesShadow + 1;
constexpr int kStatLevelTris = kStatLevelNodes + kMaxLevels;
constexpr int kStatLevelLeaves = kStatLevelTris + kMaxLevels;
constexpr int kStatLevelShaded = kStatLevelLeaves + kMaxLevels;  // counting pass: kStatShaded per level
constexpr int kStatOccluded = kStatLevelShaded + kMaxLevels;  // counting pass: occluded shadow rays
constexpr int kStatPhases = kStatOccluded + 1;  // counting pass: 2 walks x {inner, leaf, triangle} x {iterations, lanes},
                                                // then 2 walks x inner {idle, done} lanes
// counting pass, the level-1 packet walk, per wave (scalar loads: each record fetched once for the
// wave's rays): inner nodes visited, leaf records loaded, triangle records loaded
constexpr int kStatPacket = kStatPhases + 16;
constexpr int kNumStats = kStatPacket + 3;
// counting builds: per walk launch (closest / any-hit x level) and wave {start, end (100 MHz
// ticks), rays fetched, child records fetched}, after the statistics (mrt_wave_log)
constexpr int kWaveLogWaves = 8192;
constexpr int kWaveLogEntries = 2 * kMaxLevels * kWaveLogWaves * 4;

// One level of the wavefront (SoA queues).
struct Level {
    float4* rO;      // origin xyz, w = path key bits
    float4* rD;      // direction xyz, w = source primitive code bits
    uint32_t* tree;  // vertex code in the ray tree
    float4* hit;     // t, u, v, hit primitive code bits
    int4* vtx;       // material (-1 terminal), first shadow ray, first child in the next level,
                     // shadow ray count << 3 | children (1 diffuse, 2 specular, 4 transmission,
                     // stored consecutively in that order)
    float4* res;     // resolved radiance xyz, w = "intersected light" flag
    float4* sO;      // shadow ray origin, w = source primitive bits
    float4* sD;      // shadow ray direction, w = distance to the light
    float4* sC;      // light contribution Le*cos, w = occluded flag
    // textured scenes: the texel this vertex's hit wrote into its material's Kd (xyz, w = the
    // material index, -1 none), and the last such write in the vertex's subtree (Shader.cpp:112-120)
    float4* kd;
    float4* last;
    int cap;        // physical slots: kQueueSegs * segCap (level 1: its dense paths)
    int shadowCap;  // kQueueSegs * shadowSegCap
    int segCap;     // slots per segment (Queue segments above)
    int shadowSegCap;
};

// Work units: rectangles of pixels (a reference tile cut into 8-row bands).  prefix[u] is
// the first pixel slot of unit u; slots inside a unit are column-major.
struct PixelMap {
    const int4* rect;    // x0, y0, width, height
    const int* prefix;   // nUnits entries
    int nUnits;
    int pad;
};

struct RaygenArgs {
    GCamera cam;
    PixelMap map;
    const float4* tables;  // .y: the sampler table
    const float2* jitter;  // per 8-entry block b: sampler[8b + kPJitterU], sampler[8b + kPJitterV]
    int width, height;
    int slotBase;    // first pixel slot of this chunk
    int nPaths;      // slots in chunk * spp
    int spp;         // samples processed in this pass
    int sppTotal;    // samplesPixel of the renderer
    int sampleBase;  // global index of the first sample of this pass
    // the pixel sampler (Renderer's samplerPixel_): 1 StaticHaltonSeq (table draws), 0 Constant
    // (every draw constJitter); C_wrapper.cpp:144-148 picks StaticHaltonSeq iff samplesPixel > 1
    int tableJitter;
    float constJitter;
    // the level-1 packet walk generating these rays (tuning key 33): 1 also stores their records,
    // 0 leaves them to k_shade to regenerate
    int storeRays;
    int pad;
};

struct ShadeArgs {
    int maxDepth;      // RayDepthMax
    int samplesLight;  // Config::samplesLight
    float maxPoint[3]; // DepthMap::maxPoint_ (C_wrapper.cpp:79-131 maxDist)
    unsigned long long* stats;  // counting pass only (else null): kStatShaded
};

// A level's segmented queue seen as one dense index range (k_shade, k_resolve, the per-wave walk):
// dense index v -> slot g * segCap + (v - pre[g]) of the segment holding it.  Counts are clamped to
// the segment (an overflowed pass is redone).
struct SegMap {
    int pre[kQueueSegs + 1];
    int segCap;
    __device__ __forceinline__ int total() const { return pre[kQueueSegs]; }
    __device__ __forceinline__ int phys(int v) const {
        int slot = v;  // segment 0: v - pre[0]
#pragma unroll
        for (int g = 1; g < kQueueSegs; ++g)
            if (v >= pre[g]) slot = g * segCap + (v - pre[g]);
        return slot;
    }
};
__device__ __forceinline__ SegMap segMap(const int* counters, int level, bool shadows, int segCap) {
    SegMap m;
    m.segCap = segCap;
    int acc = 0;
#pragma unroll
    for (int g = 0; g < kQueueSegs; ++g) {
        m.pre[g] = acc;
        acc += min(counters[shadows ? cntShadows(level, g) : cntRays(level, g)], segCap);
    }
    m.pre[kQueueSegs] = acc;
    return m;
}
// a dense range [0, n) as segments of segCap slots: the counts of level 1 (camera rays) and of
// rays loaded from the host (mrt_trace_rays)
__device__ __forceinline__ void denseCounts(int* counters, int level, bool shadows, int n, int segCap) {
#pragma unroll
    for (int g = 0; g < kQueueSegs; ++g)
        counters[shadows ? cntShadows(level, g) : cntRays(level, g)] = max(0, min(n - g * segCap, segCap));
}

struct AccumArgs {
    PixelMap map;
    int width;
    int slotBase;
    int nSlots;
    int spp;
    int sampleBase;
    int pad;
};



void launchRaygen(const RaygenArgs& a, const Level& lv, int* counters, hipStream_t st);
// gen (level 1 with the packet walk, packetLevel1): the walk generates the camera rays itself and
// stores their records, replacing launchRaygen
bool packetLevel1(const DScene& s);
void launchTrace(const DScene& s, const Level& lv, int* counters, int level, int2* gstack, int gdepth,
                 unsigned long long* stats, bool countStats, int maxThreads, hipStream_t st,
                 const RaygenArgs* gen = nullptr);
void launchShadow(const DScene& s, const Level& lv, int* counters, int level, int2* gstack, int gdepth,
                  unsigned long long* stats, bool countStats, int maxThreads, hipStream_t st, int gridPct = 100);
// deadNext: level + 1 is the depth-capped last level (its rays are counted, never written)
// Level 1's ray generation, walk and shading in one launch (k_trace_packet_shade) where it applies
// (canFuseLevel1: DScene::fuseShade, the packet walk, Whitted / PathTracer, the lean shading, no
// counting); it replaces launchRaygen + launchTrace + launchShade of level 1.
bool canFuseLevel1(int shader, const DScene& s, const ShadeArgs& a);
void launchTraceShadeFused(int shader, const DScene& s, const Level& lv, const Level& nx, int* counters, int level,
                           const ShadeArgs& a, int2* gstack, int gdepth, int maxThreads, hipStream_t st, bool deadNext,
                           const RaygenArgs& ra);
// regen (level 1, Whitted / PathTracer): the camera rays are regenerated from *regen (cameraRay)
// instead of read from lv's records, which the packet walk then does not store
void launchShade(int shader, const DScene& s, const Level& lv, const Level& nx, int* counters, int level,
                 const ShadeArgs& a, int grid, hipStream_t st, bool deadNext = false,
                 const RaygenArgs* regen = nullptr);
// deadChildren: level + 1 is the depth-capped last level, whose results are all zero; its
// records are then not read (a zero child adds exactly nothing, section 3 of DESIGN.md)
void launchResolve(int shader, const DScene& s, const Level& lv, const Level& nx, int* counters, int level,
                   const ShadeArgs& a, int grid, hipStream_t st, bool deadChildren = false);
void launchAccumulate(const AccumArgs& a, const float4* res, int32_t* bitmap, int32_t* packed, hipStream_t st);
// level 1's resolve and the accumulation in one launch (Whitted / PathTracer; false: not launched)
bool launchResolveAccumulate(int shader, const DScene& s, const Level& lv, const Level& nx, const ShadeArgs& sa,
                             bool deadChildren, const AccumArgs& a, int32_t* bitmap, int32_t* packed, hipStream_t st);
// rank 0's frame assembly: up to kUnpackRanks shards per launch (rank first + k reads row first + k
// of the gathered array, stride entries apart)
constexpr int kUnpackRanks = 16;
struct UnpackArgs {
    PixelMap maps[kUnpackRanks];
    int n[kUnpackRanks];
    int width;
    int first;
    int stride;
    int pad;
};
void launchUnpackRanks(const UnpackArgs& a, int ranks, int maxN, const int32_t* gathered, int32_t* bitmap,
                       hipStream_t st);
void launchDumpHits(const Level& lv, int n, int32_t* kind, int32_t* index, float* t, hipStream_t st);
// hostOut (pinned host memory, kNumStats entries): the statistics copied there and the counters reset
// (and with zeroStats the statistics too), for the next chunk or pass
void launchTally(int* counters, int maxLevel, unsigned long long* stats, hipStream_t st, int skippedLevel = 0,
                 unsigned long long* hostOut = nullptr, bool zeroStats = false);
// known-answer kernels (device slab / triangle tests) and arbitrary-ray loading for tests
void launchKatSlab(const float* boxes, const float* orig, const float* dir, int n, int32_t* out, hipStream_t st);
void launchKatTriangle(const float* tris, const float* orig, const float* dir, int n, int32_t* hit, float* t,
                       hipStream_t st);
void launchLoadRays(const Level& lv, const float* orig, const float* dir, const float* dist, const uint32_t* src, int n,
                    bool any, int* counters, hipStream_t st);
int traceResidentThreadsPerCU();  // max over the trace walks of resident threads per CU
// out[2 slot], out[2 slot + 1] = real-time counter (100 MHz) before / after a spin of `ticks`
void launchSpin(unsigned long long* out, int slot, unsigned long long ticks, hipStream_t st);

}  // namespace mrt
