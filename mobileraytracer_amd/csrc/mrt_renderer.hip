// mrt_renderer.hip - the Renderer (Renderer.cpp) and desktop C-ABI (C_wrapper.cpp) of the
// MI355X render path: scene upload, wavefront queue memory, the per-frame launch sequence,
// stop / progress / ray-count bookkeeping and the exported symbols of include/mobilert_amd.h(pp).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <future>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mobilert_amd.h"
#include "mobilert_amd.hpp"
#include "mrt_kernels.hpp"
#include "mrt_scene.hpp"

namespace {

#define MRT_HIP(x)                                                                              \
    do {                                                                                        \
        const hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

thread_local std::string gLastError;

struct DeviceMem {
    std::vector<void*> ptrs;
    size_t total = 0;
    template <class T>
    T* alloc(size_t n) {
        if (n == 0) n = 1;
        void* p = nullptr;
        MRT_HIP(hipMalloc(&p, n * sizeof(T)));
        ptrs.push_back(p);
        total += n * sizeof(T);
        return static_cast<T*>(p);
    }
    template <class T>
    T* upload(const std::vector<T>& v, hipStream_t st) {
        T* p = alloc<T>(v.size());
        if (!v.empty()) MRT_HIP(hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st));
        return p;
    }
    void release() {
        for (void* p : ptrs) (void)hipFree(p);
        ptrs.clear();
        total = 0;
    }
    ~DeviceMem() { release(); }
};

// The wide collapse's node costs (toQuantizedBVH4's nodeCost).  Default (round 6): a sample of the
// frame's own rays (mrt::frameRayNodeCosts: the camera's rays, their bounces and shadow rays), so
// that the collapse minimises the wide-node visits of the rays this frame walks rather than of
// uniformly random lines: node records per shadow ray 60.6 -> 53.0, per closest-hit ray 93.0 ->
// 91.4; C4 13.94-13.97 -> 13.68-13.70 ms, N = 8 shard 2.53 -> 2.47 ms, the flat stand-in unchanged
// (profiles/r06_ray_collapse_ab.txt).  MOBILERT_COLLAPSE=area: surface areas (an empty vector);
// =greedy: round 1's greedy collapse.  Any cost gives an exact walk.
// The same sample first rotates the walk tree's BVH2 where that lowers the collapse's cost under it
// (mrt::rotateForRays, MOBILERT_RAY_ROT sweeps, default kRayRotSweeps; round 6), and the costs are
// those of the rotated tree.  Returns the tree to collapse; *cost empty: collapse by area.
#ifndef MRT_RAY_ROT_SWEEPS
#define MRT_RAY_ROT_SWEEPS 1
#endif
constexpr int kRayRotSweeps = MRT_RAY_ROT_SWEEPS;
// Renderers of one scene and camera in one process (a device group's shards, which sample the whole
// frame's rays, re-created renderers, the test suite) share the result: keyed by a 64-bit FNV-1a
// digest of everything the sample reads (the walk tree, the triangles, materials and lights, the
// camera, width, height, depth, sweeps), built once - a build in flight is waited for, as
// walkTreeOver's - and the last kFrameTreeCache kept.
constexpr size_t kFrameTreeCache = 4;
struct FrameTree {
    std::vector<mrt::HBVHNode> nodes;
    std::vector<double> cost;
};
struct Fnv64 {
    uint64_t h = 1469598103934665603ull;
    void add(const void* p, size_t n) {
        const auto* b = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    }
    template <class T>
    void pod(const T& v) { add(&v, sizeof(v)); }
};
std::vector<mrt::HBVHNode> frameWalkTree(const std::vector<mrt::HBVHNode>& wn, const mrt::HScene& sc, const mrt::GCamera& cam,
                                         int width, int height, int maxDepth, std::vector<double>* cost) {
    cost->clear();
    const char* ce = std::getenv("MOBILERT_COLLAPSE");
    if (ce != nullptr && (std::string(ce) == "area" || std::string(ce) == "greedy")) return wn;
    if (wn.empty() || sc.triangles.empty() || width <= 0 || height <= 0) {
        cost->assign(wn.size(), 0.0);
        return wn;
    }
    const char* re = std::getenv("MOBILERT_RAY_ROT");
    const int sweeps = re != nullptr ? std::atoi(re) : kRayRotSweeps;
    Fnv64 f;
    f.add(wn.data(), wn.size() * sizeof(mrt::HBVHNode));
    for (const mrt::HTriangle& t : sc.triangles) {
        f.pod(t.AC);
        f.pod(t.AB);
        f.pod(t.A);
        f.pod(t.mat);
    }
    for (const mrt::HMaterial& m : sc.materials) {
        f.pod(m.Le);
        f.pod(m.Kd);
        f.pod(m.Ks);
    }
    for (const mrt::HLight& l : sc.lights) {
        f.pod(l.kind);
        f.pod(l.tri.A);
        f.pod(l.tri.AB);
        f.pod(l.tri.AC);
    }
    f.pod(cam);
    const int dims[4] = {width, height, maxDepth, sweeps};
    f.pod(dims);
    using Entry = std::shared_ptr<const FrameTree>;
    static std::mutex mu;
    static std::unordered_map<uint64_t, std::shared_future<Entry>> cache;
    static std::deque<uint64_t> order;
    std::promise<Entry> mine;
    std::shared_future<Entry> pending;
    {
        std::lock_guard<std::mutex> lock(mu);
        const auto it = cache.find(f.h);
        if (it != cache.end()) {
            pending = it->second;
        } else {
            cache.emplace(f.h, mine.get_future().share());
            order.push_back(f.h);
            while (order.size() > kFrameTreeCache) {
                cache.erase(order.front());
                order.pop_front();
            }
        }
    }
    if (pending.valid()) {
        const Entry e = pending.get();
        *cost = e->cost;
        return e->nodes;
    }
    try {
        auto e = std::make_shared<FrameTree>();
        const std::vector<mrt::SampleRay> rays = mrt::sampleFrameRays(wn, sc, cam, maxDepth);
        e->nodes = sweeps > 0 ? mrt::rotateForRays(wn, rays, sweeps) : wn;
        e->cost = mrt::sampleRayNodeCosts(e->nodes, rays);
        mine.set_value(e);
        *cost = e->cost;
        return e->nodes;
    } catch (...) {
        mine.set_exception(std::current_exception());
        std::lock_guard<std::mutex> lock(mu);
        cache.erase(f.h);
        order.erase(std::remove(order.begin(), order.end(), f.h), order.end());
        throw;
    }
}

int bvhDepth(const std::vector<mrt::HBVHNode>& nodes) {
    if (nodes.empty()) return 0;
    int best = 0;
    std::vector<std::pair<int, int>> st{{0, 1}};
    while (!st.empty()) {
        const auto [i, d] = st.back();
        st.pop_back();
        best = std::max(best, d);
        const mrt::HBVHNode& n = nodes[static_cast<size_t>(i)];
        if (n.numPrimitives == 0 && nodes.size() > 1) {
            st.push_back({n.indexOffset, d + 1});
            st.push_back({n.indexOffset + 1, d + 1});
        }
    }
    return best;
}

float4 f4(mrt::v3 v, float w) { return make_float4(v.x, v.y, v.z, w); }
float asFloat(int32_t i) {
    float f;
    std::memcpy(&f, &i, 4);
    return f;
}

}  // namespace

// "0,1,2,3" (MOBILERT_DEVICES) -> {0, 1, 2, 3}; null or empty -> {}.  Throws on anything else.
std::vector<int32_t> mrt::parseDeviceList(const char* s) {
    std::vector<int32_t> out;
    if (s == nullptr) return out;
    std::string item;
    std::istringstream in(s);
    while (std::getline(in, item, ',')) {
        char* end = nullptr;
        const long v = std::strtol(item.c_str(), &end, 10);
        if (item.empty() || end != item.c_str() + item.size() || v < 0 || v > 0x7fffffffL)
            throw std::runtime_error(std::string("MOBILERT_DEVICES: bad ordinal '") + item + "'");
        out.push_back(static_cast<int32_t>(v));
    }
    return out;
}

namespace {

// The shard workers of a device group: one long-lived host thread per shard 1..n-1, bound to its
// shard's GPU once (hipSetDevice is per thread), woken per frame (or per sample in progressive
// mode) to run that frame's work for its shard; shard 0 runs in the calling thread.  Replaces a
// std::thread per shard and frame (creation, join and hipSetDevice on every frame).
class ShardPool {
public:
    explicit ShardPool(const std::vector<int>& devices) : n_(static_cast<int>(devices.size())), err_(devices.size()) {
        for (int i = 1; i < n_; ++i) th_.emplace_back([this, i, d = devices[static_cast<size_t>(i)]] { loop(i, d); });
    }
    ~ShardPool() {
        {
            std::lock_guard<std::mutex> lock(mu_);
            quit_ = true;
        }
        wake_.notify_all();
        for (std::thread& t : th_) t.join();
    }
    ShardPool(const ShardPool&) = delete;
    ShardPool& operator=(const ShardPool&) = delete;

    // job(i) for every shard i: 1..n-1 on the workers, 0 in the calling thread; returns when all
    // are done, then rethrows the first failure (in shard order)
    void run(const std::function<void(int)>& job) {
        std::lock_guard<std::mutex> serial(runMu_);  // one frame of the group at a time
        {
            std::lock_guard<std::mutex> lock(mu_);
            job_ = &job;
            for (std::exception_ptr& e : err_) e = nullptr;
            pending_ = n_ - 1;
            ++gen_;
        }
        wake_.notify_all();
        try {
            job(0);
        } catch (...) {
            err_[0] = std::current_exception();
        }
        {
            std::unique_lock<std::mutex> lock(mu_);
            done_.wait(lock, [this] { return pending_ == 0; });
            job_ = nullptr;
        }
        for (const std::exception_ptr& e : err_)
            if (e) std::rethrow_exception(e);
    }

private:
    void loop(int i, int device) {
        const hipError_t bound = hipSetDevice(device);
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* job = nullptr;
            {
                std::unique_lock<std::mutex> lock(mu_);
                wake_.wait(lock, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
                job = job_;
            }
            try {
                if (bound != hipSuccess)
                    throw std::runtime_error(std::string("shard worker: hipSetDevice: ") + hipGetErrorString(bound));
                (*job)(i);
            } catch (...) {
                err_[static_cast<size_t>(i)] = std::current_exception();
            }
            {
                std::lock_guard<std::mutex> lock(mu_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }

    const int n_;
    std::mutex runMu_, mu_;
    std::condition_variable wake_, done_;
    std::vector<std::thread> th_;
    std::vector<std::exception_ptr> err_;
    const std::function<void(int)>* job_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool quit_ = false;
};

}  // namespace

struct mrt_renderer {
    mrt_config cfg{};
    std::string objPath, mtlPath, camPath;
    int maxDepth = mrt::kRayDepthMaxDefault;
    int shader = mrt::kShaderWhitted;  // kShader* after the reference's switch (C_wrapper.cpp:153-193)
    int nLevels = 1;                   // wavefront levels: maxDepth + 1, or 1 for single-level shaders
    mrt::v3 maxPoint{1.0F, 1.0F, 1.0F};  // DepthMap
    // the pixel sampler: -1 as C_wrapper.cpp:144-148 (StaticHaltonSeq iff samplesPixel > 1),
    // 0 Constant(pixelConst), 1 StaticHaltonSeq (mrt_set_pixel_sampler)
    int pixelSampler = -1;
    float pixelConst = 0.5F;
    int rankIndex = 0, rankCount = 1;
    int device = 0;
    int shadowConcurrent = 0;  // the shadow stream runs beside the render stream (createShadowStream)
    int shadowTries = 0;       // shadow streams created until one did
    std::vector<hipStream_t> spareStreams;  // earlier candidates (kept: they hold their hardware queues)
    unsigned long long* spinTimes = nullptr;
    hipEvent_t joinIn = nullptr, joinOut = nullptr;  // the caller's stream <-> the render stream

    // scene
    mrt::GCamera cam{};
    mrt::DScene ds{};
    std::vector<int32_t> triOrder, planeOrder, sphereOrder;
    int64_t nTri = 0, nLights = 0, nPlanes = 0, nSpheres = 0, nMats = 0, nTriNodes = 0;
    int triDepth = 0, maxBvhDepth = 0;
    int stackNeed = 0;  // worst-case traversal stack entries over all node layouts

    // pixel units of every shard (rank r uses unitsByRank[r])
    std::vector<std::vector<int4>> unitsByRank;
    std::vector<std::vector<int>> prefixByRank;
    std::vector<mrt::PixelMap> mapByRank;
    int nSlots = 0, maxSlots = 0;

    // queues
    DeviceMem sceneMem, queueMem, frameMem;  // frameMem: bitmaps, kept when the queues are resized
    // The wavefront queues of one chunk of pixel slots, and the two streams it runs on.
    struct Pipe {
        mrt::Level levels[mrt::kMaxLevels]{};
        int* counters = nullptr;
        unsigned long long* stats = nullptr;
        int2* gstack = nullptr;        // spill stacks of the closest-hit kernel ...
        int2* gstackShadow = nullptr;  // ... and of the any-hit kernel (the two can run together)
        hipStream_t shadowStream = nullptr;  // any-hit launches, overlapped with the next level
        std::vector<hipEvent_t> syncPool;    // ordering events between the streams
        std::vector<hipEvent_t> evPool;      // profiling: 5 timing events per level and chunk
        size_t evCount = 0;
    } pipe;
    int chunkSlots = 0;
    int gdepth = 0;
    int traceThreads = 0, workGrid = 0;  // traceThreads: resident trace threads, whole device
    int cus = 0;
    int shadeGridPerCU = -1;             // tuning key 11: k_shade workgroups per CU (14: two per resident slot
                                         // of the lean kernel; 0: workGrid; -1 auto: by paths per lane)
    int32_t* dBitmap = nullptr;  // for the host-bitmap entry point
    int32_t* dBackup = nullptr;  // progressive mode: the running average before the current pass
    size_t backupN = 0;
    hipStream_t stream = nullptr;
    int overlap = 1;                     // tuning key 3: shadow rays on their own stream
    int skipLast = 1;                    // tuning key 7: no closest-hit walk for the depth-capped last level
    int shadowGridPct = 0;               // tuning key 6: shadow walk grid, percent of its occupancy grid (0 auto)
    int fuseL1Mode = -1;                 // tuning key 17: level 1 fused (1), in separate launches (0), -1 auto
    int genL1 = 2;                       // tuning key 33: the unfused level-1 packet walk generates its camera rays
                                         // (1: and stores them; 2: k_shade regenerates them; 0: k_raygen)
    int resolveAcc = 1;                  // tuning key 34: level 1's resolve and the accumulation in one launch
    int shadeWaitsShadow = 0;            // tuning key 35: shade(L) waits for shadow(L - 2) (round 1's order)
    int refill = 0;                      // tuning key 9: walk refill threshold (0 auto: by paths per lane)
    int64_t shadeLaunches = 0;           // k_shade launches of the current pass
    bool walkSkipped = false;            // the last pass skipped that walk
    bool fusedL1 = false;                // the last pass ran level 1 as k_trace_packet_shade
    int lastShadowRender = 1;            // tuning key 27: the last shadow walk on the render stream
    int walkGridCap = 0;                 // tuning key 28: at most this many workgroups per walk launch (0: none)
    unsigned long long* hostStats = nullptr;  // pinned, coherent: the per-pass statistics, written by k_tally
    // the device counters / statistics are all zero once the work enqueued so far has run (the last
    // k_tally reset them): the next pass needs no memset launch
    bool countersClean = false, statsClean = false;

    // host copies for the GL preview of the Android front end (mrt_preview_arrays; kept only for
    // renderers made by mrt_create_from_memory): triangles in BVH order and the materials
    bool keepHost = false;
    std::vector<mrt::HTriangle> hostTris;
    std::vector<mrt::HMaterial> hostMats;

    // state (Renderer.hpp:30-40)
    std::atomic<bool> stopFlag{false};
    std::atomic<int32_t> sample{0};
    std::atomic<uint64_t> totalRays{0};
    int profileFlags = 0;
    mrt_frame_stats last{};

    // device group (mrt_config.devices): this renderer is shard 0 on devices[0] and the group's
    // head; peers[i - 1] is shard i on devices[i].  Every shard renders into its own packed buffer
    // (dOwnPacked, on its device); the head gathers them into dGathered and unpacks the frame.
    std::vector<std::unique_ptr<mrt_renderer>> peers;
    int32_t* dOwnPacked = nullptr;
    int32_t* dGathered = nullptr;
    std::unique_ptr<ShardPool> shardPool;  // the head's shard workers (declared after peers: stopped first)

    ~mrt_renderer() {
        if (hostStats != nullptr) (void)hipHostFree(hostStats);
        for (hipEvent_t e : pipe.evPool) (void)hipEventDestroy(e);
        for (hipEvent_t e : pipe.syncPool) (void)hipEventDestroy(e);
        if (pipe.shadowStream != nullptr) (void)hipStreamDestroy(pipe.shadowStream);
        for (hipStream_t s : spareStreams) (void)hipStreamDestroy(s);
        if (joinIn != nullptr) (void)hipEventDestroy(joinIn);
        if (joinOut != nullptr) (void)hipEventDestroy(joinOut);
        if (stream != nullptr) (void)hipStreamDestroy(stream);
    }
};

namespace {

void buildUnits(mrt_renderer* r) {
    const int W = r->cfg.width, H = r->cfg.height;
    const int tilesPerSide = static_cast<int>(std::sqrt(static_cast<double>(mrt::kNumberOfTiles)));
    const int bx = W / tilesPerSide, by = H / tilesPerSide;  // Renderer.cpp:33-34
    if (bx <= 0 || by <= 0) throw std::runtime_error("width and height must be >= 16 (Renderer.cpp:33-38)");
    const int domainSize = (W / bx) * (H / by);
    const int resolution = W * H;
    // The reference claims the 256 tiles in a shuffled Halton order; their values are j/256,
    // so roundBlock = roundf(j/256 * domainSize) (Renderer.cpp:125).  Order is irrelevant here
    // (per-pixel sample streams), duplicates are rendered once.
    std::vector<int> blocks;
    for (int j = 0; j < mrt::kNumberOfTiles; ++j) {
        const float tile = static_cast<float>(j) / static_cast<float>(mrt::kNumberOfTiles);
        const int rb = static_cast<int>(::roundf(tile * static_cast<float>(domainSize)));
        if (std::find(blocks.begin(), blocks.end(), rb) == blocks.end()) blocks.push_back(rb);
    }
    std::vector<int4> all;
    std::vector<int> owner;  // unit (tile t, band b) -> rank (t + b) % rankCount: balances short bands
    for (size_t t = 0; t < blocks.size(); ++t) {
        const int rb = blocks[t];
        const int pixel = rb * bx % resolution;               // Renderer.cpp:126
        const int startY = ((pixel / W) * by) % H;            // :127
        const int startX = pixel % W;                         // :133 ((pixel + y*W) % W)
        for (int b = 0; b * 8 < by; ++b) {
            int h = std::min(8, by - 8 * b);
            const int y0 = startY + 8 * b;
            while (h > 0 && (y0 + h - 1) * W + startX + bx - 1 >= resolution) --h;  // stay inside the bitmap
            if (h > 0) {
                all.push_back(make_int4(startX, y0, bx, h));
                owner.push_back(static_cast<int>((t + static_cast<size_t>(b)) % static_cast<size_t>(r->rankCount)));
            }
        }
    }
    r->unitsByRank.assign(static_cast<size_t>(r->rankCount), {});
    r->prefixByRank.assign(static_cast<size_t>(r->rankCount), {});
    for (size_t u = 0; u < all.size(); ++u) r->unitsByRank[static_cast<size_t>(owner[u])].push_back(all[u]);
    r->maxSlots = 0;
    for (int k = 0; k < r->rankCount; ++k) {
        int acc = 0;
        for (const int4& u : r->unitsByRank[static_cast<size_t>(k)]) {
            r->prefixByRank[static_cast<size_t>(k)].push_back(acc);
            acc += u.z * u.w;
        }
        if (k == r->rankIndex) r->nSlots = acc;
        r->maxSlots = std::max(r->maxSlots, acc);
    }
    r->mapByRank.clear();
    for (int k = 0; k < r->rankCount; ++k) {
        mrt::PixelMap m{};
        m.rect = r->sceneMem.upload(r->unitsByRank[static_cast<size_t>(k)], r->stream);
        m.prefix = r->sceneMem.upload(r->prefixByRank[static_cast<size_t>(k)], r->stream);
        m.nUnits = static_cast<int>(r->unitsByRank[static_cast<size_t>(k)].size());
        r->mapByRank.push_back(m);
    }
}

void slotToXYHost(const std::vector<int4>& units, const std::vector<int>& prefix, int slot, int* x, int* y) {
    const auto it = std::upper_bound(prefix.begin(), prefix.end(), slot);
    const size_t u = static_cast<size_t>(it - prefix.begin()) - 1;
    const int off = slot - prefix[u];
    *x = units[u].x + off / units[u].w;
    *y = units[u].y + off % units[u].w;
}

void uploadScene(mrt_renderer* r, mrt::HScene& sc) {
    using namespace mrt;
    hipStream_t st = r->stream;
    std::vector<HBVHNode> pn = buildBVH(&sc.planes, &r->planeOrder);
    std::vector<HBVHNode> sn = buildBVH(&sc.spheres, &r->sphereOrder);
    std::vector<HBVHNode> tn = buildBVH(&sc.triangles, &r->triOrder);
    // the walk tree: the reference leaves regrouped by a full-sweep SAH (rebuildOverLeaves; the
    // reference tree itself with MOBILERT_WALK_TREE=0).  Rays with a non-finite 1/d and the
    // per-wave reference walk use the reference tree, appended after it in the same node array.
    // ... rotated for the frame's ray sample, whose node costs the wide collapse below uses
    std::vector<double> rayCost;
    const std::vector<HBVHNode> wn =
        frameWalkTree(walkTreeOver(tn), sc, r->cam, r->cfg.width, r->cfg.height, r->maxDepth, &rayCost);
    r->nTri = static_cast<int64_t>(sc.triangles.size());
    r->nPlanes = static_cast<int64_t>(sc.planes.size());
    r->nSpheres = static_cast<int64_t>(sc.spheres.size());
    r->nLights = static_cast<int64_t>(sc.lights.size());
    r->nMats = static_cast<int64_t>(sc.materials.size());
    r->nTriNodes = static_cast<int64_t>(tn.size());
    r->triDepth = std::max(bvhDepth(tn), bvhDepth(wn));
    r->maxBvhDepth = std::max({r->triDepth, bvhDepth(pn), bvhDepth(sn)});
    r->stackNeed = r->maxBvhDepth + 2;

    if (r->keepHost) {
        r->hostTris = sc.triangles;  // BVH order, as Shader::getTriangles returns them
        r->hostMats = sc.materials;
    }
    std::vector<GNode> g;
    DScene& d = r->ds;
    // cull words (certified mode) for the reference tree only: that mode walks it for every ray
    const std::vector<uint32_t> conesRef = triangleConeWords(tn, sc.triangles);
    // the walk tree, numbered (top breadth-first), then quantized; the reference tree in its own
    // GNode array
    std::vector<QNode4> qn;
    d.qEnabled = toQuantizedBVH4(wn, sc.triangles.size(), &d.triRoot, kTopNodesMax, &d.triTop, &d.qgrid, &qn, nullptr,
                                 rayCost.empty() ? nullptr : &rayCost) ? 1 : 0;
    if (d.qEnabled == 0 || qn.empty()) qn.resize(1);  // (a leaf or empty root: no inner node)
    d.triQNodes = r->sceneMem.upload(qn, st);
    {
        // the packet walk's copy: float(q) is exact (q < 2^16), so its planes fma(q, qa, qb) are
        // the per-lane walk's bit for bit, without a conversion per bound (its loads are scalar:
        // twice the bytes cost nothing there)
        static_assert(kWalkWidth == 4, "packet nodes: 4 children");
        std::vector<float> qf(32 * qn.size(), 0.0F);
        for (size_t k = 0; k < qn.size(); ++k) {
            const QNode4& q = qn[k];
            for (int c = 0; c < kWalkWidth; ++c) {
                const uint32_t w0 = q.q[3 * c], w1 = q.q[3 * c + 1], w2 = q.q[3 * c + 2];
                // (min xyz, max xyz) from the per-axis words min | max << 16
                const uint32_t v[6] = {w0 & 0xFFFFu, w1 & 0xFFFFu, w2 & 0xFFFFu, w0 >> 16, w1 >> 16, w2 >> 16};
                for (int j = 0; j < 6; ++j) qf[32 * k + 6 * static_cast<size_t>(c) + static_cast<size_t>(j)] = static_cast<float>(v[j]);
                std::memcpy(&qf[32 * k + 24 + static_cast<size_t>(c)], &q.ref[c], sizeof(int32_t));
            }
        }
        d.triQNodesF = r->sceneMem.upload(qf, st);
    }
    // a visit pushes up to kWalkWidth - 1 entries: the walk's stack holds that many per level
    {
        int depth4 = 0;
        std::vector<std::pair<int32_t, int>> w;
        if (d.qEnabled != 0 && d.triRoot.count > 0 && d.triRoot.ref >= 0) w.push_back({d.triRoot.ref, 1});
        while (!w.empty()) {
            const auto [i, dep] = w.back();
            w.pop_back();
            depth4 = std::max(depth4, dep);
            for (int32_t c : qn[static_cast<size_t>(i)].ref)
                if (c >= 0 && c != kEmptyChild) w.push_back({c, dep + 1});
        }
        r->stackNeed = std::max(r->stackNeed, (kWalkWidth - 1) * depth4 + 2);
    }
    toDeviceBVH(tn, sc.triangles.size(), &g, &d.triRootRef, 0, nullptr, &conesRef);
    {
        // per leaf (indexed by its first triangle, 48 B): the exact reference box, then the
        // certified-cull record of its own triangles (leafCullRecord) for the exact mode
        std::vector<float4> lb(std::max<size_t>(1, 3 * sc.triangles.size()), make_float4(0.0F, 0.0F, 0.0F, 0.0F));
        for (const HBVHNode& n : tn) {
            if (n.numPrimitives <= 0) continue;
            const size_t f = static_cast<size_t>(n.indexOffset);
            float c[6];
            leafCullRecord(sc.triangles, f, f + static_cast<size_t>(n.numPrimitives), n.box, c);
            lb[3 * f] = make_float4(n.box.mn.x, n.box.mn.y, n.box.mn.z, n.box.mx.x);
            lb[3 * f + 1] = make_float4(n.box.mx.y, n.box.mx.z, c[0], c[1]);
            lb[3 * f + 2] = make_float4(c[2], c[3], c[4], c[5]);
        }
        d.leafBoxes = r->sceneMem.upload(lb, st);
    }
    d.triNodes = r->sceneMem.upload(g, st);
    toDeviceBVH(pn, sc.planes.size(), &g, &d.planeRoot);
    d.planeNodes = r->sceneMem.upload(g, st);
    toDeviceBVH(sn, sc.spheres.size(), &g, &d.sphereRoot);
    d.sphereNodes = r->sceneMem.upload(g, st);

    std::vector<float4> v;
    v.reserve(sc.triangles.size() * 3);
    for (const HTriangle& t : sc.triangles) {
        v.push_back(f4(t.A, 0.0F));
        v.push_back(f4(t.AB, 0.0F));
        v.push_back(f4(t.AC, 0.0F));
    }
    d.triGeom = r->sceneMem.upload(v, st);
    v.clear();
    for (const HTriangle& t : sc.triangles) {
        v.push_back(f4(t.nA, asFloat(t.mat)));
        v.push_back(f4(t.nB, 0.0F));
        v.push_back(f4(t.nC, 0.0F));
    }
    d.triShade = r->sceneMem.upload(v, st);
    v.clear();
    // the 16-B head of each shading record (what k_shade gathers first): nA and
    // ((material + 1) << 1 | flat), flat when the three normals are the same bits (every
    // triangle of an OBJ without normals, OBJLoader.cpp:175-181), so nB and nC are not read
    for (const HTriangle& t : sc.triangles) {
        const bool flat = std::memcmp(&t.nA, &t.nB, sizeof(t.nA)) == 0 && std::memcmp(&t.nA, &t.nC, sizeof(t.nA)) == 0;
        v.push_back(f4(t.nA, asFloat(static_cast<int32_t>((static_cast<uint32_t>(t.mat + 1) << 1) | (flat ? 1u : 0u)))));
    }
    d.triHead = r->sceneMem.upload(v, st);
    v.clear();
    // textures: triangle texture coordinates, texture table and texels (textured scenes only)
    d.textured = 0;
    for (const HMaterial& m : sc.materials) d.textured |= (m.texId >= 0 && !sc.textures.empty()) ? 1 : 0;
    if (d.textured != 0) {
        for (const HTriangle& t : sc.triangles) {
            v.push_back(make_float4(t.tA.x, t.tA.y, t.tB.x, t.tB.y));
            v.push_back(make_float4(t.tC.x, t.tC.y, 0.0F, 0.0F));
        }
        d.triTex = r->sceneMem.upload(v, st);
        v.clear();
        std::vector<int4> info;
        std::vector<uint8_t> bytes;
        for (const HTexture& t : sc.textures) {
            info.push_back(make_int4(t.width, t.height, t.channels, static_cast<int>(bytes.size())));
            bytes.insert(bytes.end(), t.texels.begin(), t.texels.end());
        }
        d.texInfo = r->sceneMem.upload(info, st);
        d.texels = r->sceneMem.upload(bytes, st);
    } else {
        d.triTex = nullptr;
        d.texInfo = nullptr;
        d.texels = nullptr;
    }
    for (const HPlane& p : sc.planes) {
        v.push_back(f4(p.normal, asFloat(p.mat)));
        v.push_back(f4(p.point, 0.0F));
    }
    d.planes = r->sceneMem.upload(v, st);
    v.clear();
    for (const HSphere& s : sc.spheres) {
        v.push_back(f4(s.center, s.sqRadius));
        v.push_back(make_float4(asFloat(s.mat), 0.0F, 0.0F, 0.0F));
    }
    d.spheres = r->sceneMem.upload(v, st);
    v.clear();
    for (const HLight& l : sc.lights) {
        if (l.kind == kAreaLight) {
            v.push_back(f4(l.tri.A, asFloat(1)));
            v.push_back(f4(l.tri.AB, 0.0F));
            v.push_back(f4(l.tri.AC, 0.0F));
        } else {
            v.push_back(f4(l.position, asFloat(0)));
            v.push_back(make_float4(0, 0, 0, 0));
            v.push_back(make_float4(0, 0, 0, 0));
        }
        // w: the index of the light's own material (Light::radiance_, appended after the scene's):
        // a hit on an area light carries that material (AreaLight.cpp:32-41), whose Kd / Ks / Kt
        // DiffuseMaterial reads (DiffuseMaterial.cpp:12-28)
        v.push_back(f4(l.radiance.Le, asFloat(static_cast<int32_t>(sc.materials.size() + (&l - sc.lights.data())))));
    }
    d.lights = r->sceneMem.upload(v, st);
    v.clear();
    std::vector<HMaterial> allMats = sc.materials;
    for (const HLight& l : sc.lights) allMats.push_back(l.radiance);
    for (const HMaterial& m : allMats) {
        v.push_back(f4(m.Le, m.ior));
        v.push_back(f4(m.Kd, asFloat(m.texId)));  // w: texture index (-1 none)
        v.push_back(f4(m.Ks, 0.0F));
        v.push_back(f4(m.Kt, 0.0F));
    }
    d.mats = r->sceneMem.upload(v, st);
    // Naive (accelerator 1): the BVH-order index of each primitive in input order
    d.accel = r->cfg.accelerator;
    auto inverse = [](const std::vector<int32_t>& order) {
        std::vector<int32_t> inv(std::max<size_t>(order.size(), 1), 0);
        for (size_t j = 0; j < order.size(); ++j) inv[static_cast<size_t>(order[j])] = static_cast<int32_t>(j);
        return inv;
    };
    d.triNaive = r->sceneMem.upload(inverse(r->triOrder), st);
    d.planeNaive = r->sceneMem.upload(inverse(r->planeOrder), st);
    d.sphereNaive = r->sceneMem.upload(inverse(r->sphereOrder), st);
    // RegularGrid (accelerator 2): one 32^3 grid per primitive kind (Shader.cpp:56-61)
    auto gridOf = [&](const HGrid& h) {
        GGrid gg{};
        const v3 m = h.world.mn;
        const float mnv[3] = {m.x, m.y, m.z}, csv[3] = {h.cellSize.x, h.cellSize.y, h.cellSize.z},
                    csiv[3] = {h.cellSizeInv.x, h.cellSizeInv.y, h.cellSizeInv.z};
        for (int a = 0; a < 3; ++a) {
            gg.mn[a] = mnv[a];
            gg.cs[a] = csv[a];
            gg.csi[a] = csiv[a];
        }
        gg.count = h.count;
        gg.start = r->sceneMem.upload(h.start, st);
        gg.items = r->sceneMem.upload(h.items.empty() ? std::vector<int32_t>(1, 0) : h.items, st);
        return gg;
    };
    d.planeGrid = GGrid{};
    d.sphereGrid = GGrid{};
    d.triGrid = GGrid{};
    if (d.accel == kAccGrid) {
        d.planeGrid = gridOf(buildGrid(sc.planes, r->planeOrder));
        d.sphereGrid = gridOf(buildGrid(sc.spheres, r->sphereOrder));
        d.triGrid = gridOf(buildGrid(sc.triangles, r->triOrder));
    }
    d.nLights = static_cast<int32_t>(sc.lights.size());
    d.nMats = static_cast<int32_t>(sc.materials.size());
    d.cull = r->cfg.cull;
    d.variant = kDefaultTraceVariant;
    // the depth-capped last level's children count as absent in the resolve only while no
    // material coefficient is infinite or NaN (inf * 0 would be NaN in the reference)
    d.anyOrder = 1;
    d.tailDonate = 1;
    d.refill = 32;  // kWalkRefill
    d.leanShade = 1;
    d.packet = r->stackNeed <= kPacketStack ? 1 : 0;  // the packet walk's uniform stack must hold the tree's need
    // level 1 fused or not: chosen per pass by paths per walk lane (tuning key 17, renderPass)
    d.fuseShade = 0;
    d.matsFinite = 1;
    for (const HMaterial& m : sc.materials) {
        for (const v3 c : {m.Kd, m.Ks, m.Kt})
            if (!std::isfinite(c.x) || !std::isfinite(c.y) || !std::isfinite(c.z)) d.matsFinite = 0;
    }

    // the sample tables interleaved with the hemisphere's cos / sin: one vertex's draws
    // (consecutive indices from an 8-aligned start) are one 128-byte line
    std::vector<float> shaderT, samplerT, trig;
    fillHaltonTable(&shaderT, kSeedShaderTable);
    fillHaltonTable(&samplerT, kSeedSamplerTable);
    fillHemisphereTrig(shaderT, &trig);
    std::vector<float4> tab(shaderT.size());
    for (size_t k = 0; k < shaderT.size(); ++k) tab[k] = make_float4(shaderT[k], samplerT[k], trig[2 * k], trig[2 * k + 1]);
    d.tables = r->sceneMem.upload(tab, st);
    std::vector<float4> draws(2 * (tab.size() / 8));
    for (size_t b = 0; b < tab.size() / 8; ++b) {
        const float4* e = tab.data() + 8 * b;
        draws[2 * b] = make_float4(e[kPRussian].y, e[kPHemi1].z, e[kPHemi1].w, e[kPHemi2].x);
        draws[2 * b + 1] = make_float4(e[purposeLightPick(0)].x, e[purposeLightR(0)].y, e[purposeLightS(0)].y, 0.0F);
    }
    d.vertexDraws = r->sceneMem.upload(draws, st);
    std::vector<float2> jit(tab.size() / 8);
    for (size_t b = 0; b < jit.size(); ++b) jit[b] = make_float2(tab[8 * b + kPJitterU].y, tab[8 * b + kPJitterV].y);
    d.jitterDraws = r->sceneMem.upload(jit, st);
    MRT_HIP(hipStreamSynchronize(st));
}

void setPixelSampler(const mrt_renderer* r, mrt::RaygenArgs* ra) {
    ra->tableJitter = r->pixelSampler < 0 ? (r->cfg.samplesPixel > 1 ? 1 : 0) : r->pixelSampler;
    ra->constJitter = r->pixelSampler == 0 ? r->pixelConst : 0.5F;
}

void allocQueues(mrt_renderer* r, int chunkSlots, int growth) {
    using namespace mrt;
    r->queueMem.release();
    const int spp = std::max(1, r->cfg.samplesPixel);
    const int spl = std::max(1, r->cfg.samplesLight);
    r->chunkSlots = chunkSlots;
    const size_t n1 = static_cast<size_t>(chunkSlots) * static_cast<size_t>(spp);
    const size_t capN = n1 * static_cast<size_t>(growth);
    const int nLevels = r->nLevels;
    r->gdepth = std::max(1, r->stackNeed - kLdsStackMin);
    mrt_renderer::Pipe& pp = r->pipe;
    // Ray / hit / payload buffers of levels L and L+2 are never live together (level L's rays are
    // dead once k_shade(L) has read them; its vertex and result records stay until the resolve),
    // but one set per level keeps the shadow stream's overlap free of reuse hazards.
    for (int l = 1; l <= nLevels + 1 && l < kMaxLevels; ++l) {
        Level& lv = pp.levels[l];
        const bool real = l <= nLevels;
        // Queue segments (mrt_kernels.hpp): level 1 is its dense paths cut into kQueueSegs pieces;
        // a deeper level's segments each hold an eighth of the level's rays plus slack for the uneven
        // split over the shading workgroups (an overflow re-renders with smaller chunks, as before)
        size_t segCap, shadowSegCap;
        if (kQueueSegs == 1) {
            segCap = (l == 1) ? n1 : capN;
            shadowSegCap = segCap * spl;
        } else if (l == 1) {
            segCap = (n1 + kQueueSegs - 1) / kQueueSegs;
            shadowSegCap = (n1 * spl * 5 / 4 + kQueueSegs - 1) / kQueueSegs + static_cast<size_t>(spl) * 4 * 256;
        } else {
            segCap = (capN * 5 / 4 + kQueueSegs - 1) / kQueueSegs + 3 * 4 * 256;
            shadowSegCap = (capN * spl * 5 / 4 + kQueueSegs - 1) / kQueueSegs + static_cast<size_t>(spl) * 4 * 256;
        }
        const size_t cap = segCap * kQueueSegs;
        lv = Level{};
        lv.cap = real ? static_cast<int>(cap) : 0;
        lv.shadowCap = real ? static_cast<int>(shadowSegCap * kQueueSegs) : 0;
        lv.segCap = real ? static_cast<int>(segCap) : 0;
        lv.shadowSegCap = real ? static_cast<int>(shadowSegCap) : 0;
        const size_t rays = real ? cap : 0;  // level nLevels + 1: no rays (its parents are terminal)
        lv.rO = r->queueMem.alloc<float4>(rays);
        lv.rD = r->queueMem.alloc<float4>(rays);
        lv.tree = r->queueMem.alloc<uint32_t>(rays);
        lv.hit = r->queueMem.alloc<float4>(rays);
        if (real) {
            lv.sO = r->queueMem.alloc<float4>(shadowSegCap * kQueueSegs);
            lv.sD = r->queueMem.alloc<float4>(shadowSegCap * kQueueSegs);
            lv.vtx = r->queueMem.alloc<int4>(cap);
            lv.res = r->queueMem.alloc<float4>(cap);
            lv.sC = r->queueMem.alloc<float4>(shadowSegCap * kQueueSegs);
        }
        const bool tex = real && r->ds.textured != 0;
        lv.kd = tex ? r->queueMem.alloc<float4>(cap) : nullptr;
        lv.last = tex ? r->queueMem.alloc<float4>(cap) : nullptr;
    }
    pp.counters = r->queueMem.alloc<int>(kNumCounters);
    pp.stats = r->queueMem.alloc<unsigned long long>(kNumStats + kWaveLogEntries);
    r->countersClean = r->statsClean = false;  // (fresh allocations: not zeroed)
    pp.gstack = r->queueMem.alloc<int2>(static_cast<size_t>(r->traceThreads) * static_cast<size_t>(r->gdepth));
    pp.gstackShadow = r->queueMem.alloc<int2>(static_cast<size_t>(r->traceThreads) * static_cast<size_t>(r->gdepth));
}

// Whether kernels launched on streams a and b run at the same time: two bounded spins, one per
// stream, overlap in time iff the streams feed different hardware queues.
bool streamsConcurrent(mrt_renderer* r, hipStream_t a, hipStream_t b) {
    if (r->spinTimes == nullptr) r->spinTimes = r->sceneMem.alloc<unsigned long long>(4);
    unsigned long long h[4] = {};
    for (int round = 0; round < 2; ++round) {  // round 0 warms the queues up (created on first use)
        mrt::launchSpin(r->spinTimes, 0, round == 0 ? 100 : 20000, a);  // 200 us
        mrt::launchSpin(r->spinTimes, 1, round == 0 ? 100 : 20000, b);
        MRT_HIP(hipStreamSynchronize(a));
        MRT_HIP(hipStreamSynchronize(b));
    }
    MRT_HIP(hipMemcpy(h, r->spinTimes, sizeof(h), hipMemcpyDeviceToHost));
    return h[2] < h[1] && h[0] < h[3];
}

// The render chain runs on the renderer's own stream, the shadow walks on a second one, joined to
// the caller's stream by events.  HIP maps a process's streams onto a few hardware queues
// (GPU_MAX_HW_QUEUES, 4 by default, shared least-used); two streams on one queue run their kernels
// one after the other, and the shadow walk of level L no longer overlaps level L + 1 (one rank's C4
// shard at N = 8: 2.96 -> 3.80 ms with three streams of the front end created before the renderer,
// DESIGN.md section 6).  So the pair is checked at creation with two timed spins, and the shadow
// stream is created again (the earlier ones kept: they hold their queues) until the two run
// concurrently; after kMaxShadowStreams tries the shadow walks are serialised on the render stream
// (mrt_scene_info.shadowStreamConcurrent = 0).
constexpr int kMaxShadowStreams = 8;
void createShadowStream(mrt_renderer* r) {
    for (int k = 0; k < kMaxShadowStreams; ++k) {
        hipStream_t s = nullptr;
        MRT_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        if (r->pipe.shadowStream != nullptr) r->spareStreams.push_back(r->pipe.shadowStream);
        r->pipe.shadowStream = s;
        r->shadowTries = k + 1;
        if (streamsConcurrent(r, r->stream, s)) {
            r->shadowConcurrent = 1;
            return;
        }
    }
    r->shadowConcurrent = 0;
    r->overlap = 0;
}

// Chunk size: every slot of the shard in one pass, within the path budget.
int chunkFor(const mrt_renderer* r) {
    const size_t spp = static_cast<size_t>(std::max(1, r->cfg.samplesPixel));
    const size_t maxPaths = r->cfg.maxPathsPerPass > 0 ? static_cast<size_t>(r->cfg.maxPathsPerPass) : (size_t{1} << 24);
    return static_cast<int>(std::max<size_t>(1, std::min(static_cast<size_t>(r->nSlots), maxPaths / spp)));
}

hipEvent_t syncEvent(mrt_renderer::Pipe& p, size_t i) {
    while (p.syncPool.size() <= i) {
        hipEvent_t e;
        MRT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        p.syncPool.push_back(e);
    }
    return p.syncPool[i];
}

hipEvent_t poolEvent(mrt_renderer::Pipe& p) {
    const size_t i = p.evCount++;
    while (p.evPool.size() <= i) {
        hipEvent_t e;
        MRT_HIP(hipEventCreate(&e));
        p.evPool.push_back(e);
    }
    return p.evPool[i];
}

// One pass over this shard's pixel slots: samples [sampleBase, sampleBase + spp).
void renderPass(mrt_renderer* r, int32_t* dBitmap, int32_t* dPacked, hipStream_t st, int sampleBase, int spp) {
    using namespace mrt;
    const int shader = r->shader;
    const bool timing = (r->profileFlags & 1) != 0;
    const bool counting = (r->profileFlags & 2) != 0;
    mrt_renderer::Pipe& pp = r->pipe;
    const int spl = std::max(1, r->cfg.samplesLight);
    ShadeArgs sa{r->maxDepth, spl, {r->maxPoint.x, r->maxPoint.y, r->maxPoint.z}, counting ? pp.stats : nullptr};
    const int nLevels = r->nLevels;
    const mrt::PixelMap& map = r->mapByRank[static_cast<size_t>(r->rankIndex)];
    if (!r->statsClean || counting)
        MRT_HIP(hipMemsetAsync(pp.stats, 0, sizeof(unsigned long long) * (kNumStats + (counting ? kWaveLogEntries : 0)), st));
    r->statsClean = false;
    if (r->hostStats == nullptr)
        MRT_HIP(hipHostMalloc(&r->hostStats, sizeof(unsigned long long) * kNumStats, hipHostMallocCoherent));
    std::memset(r->hostStats, 0, sizeof(unsigned long long) * kNumStats);  // (no chunk run: zeros)
    pp.evCount = 0;
    r->shadeLaunches = 0;
    // Any-hit (shadow) rays of level L run on a second stream, overlapped with the closest-hit
    // trace and shading of level L+1: the persistent kernels' drain phases fill each other.
    // Orders: shade(L) -> shadow(L); shadow(L) -> shade(L+2) (shade(L+2) rewrites level L+2's
    // shadow queue only, but the walk kernels share nothing else, so the order is for the spill
    // stacks' sake: one per kernel kind); every shadow(L) -> resolve.
    hipStream_t sb = r->overlap == 1 && r->shadowConcurrent != 0 ? pp.shadowStream : st;
    // The last level (depth RayDepthMax + 1) shades to zero whatever its rays hit: shade()
    // returns at the depth cap (PathTracer.cpp:24-26, Whitted.cpp:15-17), so its closest-hit
    // walk is dead work and is skipped.  Not for textured scenes (rayTrace writes the texel Kd
    // before shade() returns, Shader.cpp:114-122).
    const bool skipLast = r->skipLast != 0 && r->ds.textured == 0 &&
                          (shader == kShaderWhitted || shader == kShaderPathTracer) && nLevels > r->maxDepth;
    r->walkSkipped = skipLast;
    // ... and with it the level's shading (every record terminal, radiance 0) and resolve: the
    // parents' resolve treats the capped children as absent, which gives the same bits while
    // every material is finite (Ks * 0 and Kd * 0 added to sums that start at +0), and the
    // parents write no payload for them (only their count)
    const bool skipLastShade = skipLast && nLevels >= 2 && r->ds.matsFinite != 0;
    for (int slot0 = 0; slot0 < r->nSlots && !r->stopFlag.load(); slot0 += r->chunkSlots) {
        const int nChunk = std::min(r->chunkSlots, r->nSlots - slot0);
        if (!r->countersClean) MRT_HIP(hipMemsetAsync(pp.counters, 0, sizeof(int) * kNumCounters, st));
        r->countersClean = false;
        RaygenArgs ra{};
        ra.cam = r->cam;
        ra.map = map;
        ra.tables = r->ds.tables;
        ra.jitter = r->ds.jitterDraws;
        ra.width = r->cfg.width;
        ra.height = r->cfg.height;
        ra.slotBase = slot0;
        ra.nPaths = nChunk * spp;
        ra.spp = spp;
        ra.sppTotal = r->cfg.samplesPixel;
        setPixelSampler(r, &ra);
        ra.sampleBase = sampleBase;
        // With few paths per resident walk lane (a small shard: C4 at N >= 4) the levels are short
        // and tail-bound, and a full-width shadow walk starves the next level's shading of CUs;
        // a narrower shadow grid leaves them room (C4 shard at N = 8: 2.92 -> 2.83 ms; at N = 1 the
        // full grid is 2.6 % faster).  Results do not depend on the grid.
        const double pathsPerLane = static_cast<double>(ra.nPaths) / std::max(1, r->traceThreads);
        // Level 1 fused (ray generation, packet walk and shading in one launch, tuning key 17) where
        // it applies; by default below 12 paths per resident walk lane (traceThreads: the packet
        // walk's 8 workgroups per CU): C4 at N = 2 (7.9 paths per lane) 7.59 -> 7.44 ms, at N = 4 / 8
        // the same, at N = 1 (15.8) separate launches are faster, 13.94 vs 14.09 ms
        // (profiles/r06_fused_level1_ab.txt).  (With per-launch events too: the serialised roofline
        // frames time the kernel the timed frames run.)
        r->ds.fuseShade = r->fuseL1Mode >= 0 ? r->fuseL1Mode : (pathsPerLane < 12.0 ? 1 : 0);
        const bool fuseL1 = nLevels >= 1 && !(skipLast && nLevels == 1) && !(skipLastShade && nLevels == 1) &&
                            canFuseLevel1(shader, r->ds, sa);
        r->fusedL1 = fuseL1;
        // Unfused, the packet walk generates the camera rays and stores the records k_shade reads
        // (tuning key 33): no k_raygen launch, no ray reads in the walk
        const bool genL1 = !fuseL1 && r->genL1 != 0 && nLevels >= 1 && !(skipLast && nLevels == 1) &&
                           packetLevel1(r->ds);
        // ... and with key 33 = 2 k_shade regenerates them instead of reading stored records
        const bool regenL1 = genL1 && r->genL1 == 2 && (shader == kShaderWhitted || shader == kShaderPathTracer) &&
                             !(skipLastShade && nLevels == 1);
        ra.storeRays = regenL1 ? 0 : 1;
        if (!fuseL1 && !genL1) launchRaygen(ra, pp.levels[1], pp.counters, st);
        // the walk launches' thread cap (tuning key 28 narrows it; the spill stacks hold traceThreads)
        const int walkThreads = r->walkGridCap > 0 ? std::min(r->traceThreads, r->walkGridCap * kBlock)
                                                   : r->traceThreads;
        // (round 2, 4-wide walk tree: C4 shard at N = 8 60 / 50 % -> 2.55 / 2.50 ms; N = 1 100 / 80 /
        // 70 % with 28 shading workgroups per CU -> 13.48 / 13.34 / 13.34 ms).  With shadow rays on
        // the render stream (key 3 = 0) nothing runs beside the shadow walk: full grid.
        const int shadowPct = r->shadowGridPct > 0 ? r->shadowGridPct
                              : sb == st            ? 100
                              : pathsPerLane < 4.0  ? 50
                              : pathsPerLane < 8.0  ? 75
                                                    : 70;
        // k_shade's grid: 14 workgroups per CU.  (Round 2: 28 where a lane sees >= 4 paths, N = 1
        // 13.55 / 13.48 ms at 14 / 28; round 3, with the materials in LDS and the 16-B shading
        // record head, 14 everywhere: N = 1 15.47 / 15.53 ms, 20 / 36: 15.52 / 15.54 ms.)
        const int shadePerCU = r->shadeGridPerCU >= 0 ? r->shadeGridPerCU : 14;
        // refill threshold: larger batches where a lane sees few paths (a small shard: the tail
        // dominates; C4 shard at N = 8: 24 / 32 / 40 -> 2.68 / 2.64 / 2.61 ms), smaller where it
        // sees many (N = 1: 13.77 / 13.86 / 13.88 ms)
        // (re-tuned in round 3 with the walk's phase exits: N = 8 40 / 48 / 56 -> 3.17 / 3.07 /
        // 3.14 ms; N = 1 24 / 32 / 36 -> 16.60 / 16.52 / 16.54 ms)
        r->ds.refill = r->refill > 0 ? r->refill : pathsPerLane < 4.0 ? 48 : 32;
        size_t sync = 0;
        hipEvent_t shadowDone[kMaxLevels + 1] = {};
        // The last shadow walk (level nLevels - 1) runs on the render stream, right after its
        // level's shading and before the resolves that wait for it: no cross-stream hand-off at
        // either end (each cost 15-30 us on the critical path, profiles/r04_frame_timeline_*).  It
        // uses the closest-hit spill stacks, idle from then on (the depth-capped last level's walk
        // is skipped, or follows it on the same stream), so it may overlap the previous level's
        // shadow walk, still running on the shadow stream.
        const bool lastOnRender = r->lastShadowRender != 0 && sb != st && nLevels >= 2;
        // (No event orders the shadow stream after the render stream's earlier work: every shadow
        // launch waits for its level's shading, recorded on the render stream, and the previous
        // chunk's shadow walks all finished before its resolves.  Round 6 dropped that marker, one
        // event packet before each pass's first kernel.)
        for (int l = 1; l <= nLevels; ++l) {
            if (timing) MRT_HIP(hipEventRecord(poolEvent(pp), st));
            // level 1 without per-launch events or counting: the packet walk generates its camera rays
            // and shades its own hits
            const bool fused = fuseL1 && l == 1;
            if (fused) {
                launchTraceShadeFused(shader, r->ds, pp.levels[l], pp.levels[l + 1], pp.counters, l, sa, pp.gstack,
                                      r->gdepth, walkThreads, st, skipLastShade && l + 1 == nLevels, ra);
                ++r->shadeLaunches;
            }
            if (!fused && !(skipLast && l == nLevels))
                launchTrace(r->ds, pp.levels[l], pp.counters, l, pp.gstack, r->gdepth, pp.stats, counting,
                            walkThreads, st, genL1 && l == 1 ? &ra : nullptr);
            if (timing) MRT_HIP(hipEventRecord(poolEvent(pp), st));
            // (round 1's shadow queues alternated by level parity, so shade(L) waited for shadow(L - 2);
            // every level has its own queues since, and the wait - an event packet, ~6 us of command
            // processing on the critical path - only with tuning key 35 = 1)
            if (r->shadeWaitsShadow != 0 && sb != st && l >= 3) MRT_HIP(hipStreamWaitEvent(st, shadowDone[l - 2], 0));
            const bool onRender = lastOnRender && l + 1 >= nLevels;  // the last shadow walk, and the level after it
            const hipStream_t ss = onRender ? st : sb;
            if (!fused && !(skipLastShade && l == nLevels)) {
                launchShade(shader, r->ds, pp.levels[l], pp.levels[l + 1], pp.counters, l, sa,
                            shadePerCU > 0 ? r->cus * shadePerCU : r->workGrid, st,
                            skipLastShade && l + 1 == nLevels, regenL1 && l == 1 ? &ra : nullptr);
                ++r->shadeLaunches;
            }
            if (timing) MRT_HIP(hipEventRecord(poolEvent(pp), st));
            // (the hand-off event completed by k_shade's own launch - hipExtLaunchKernel's stop event -
            // instead of this marker measured the same: the ~5 us before the next walk stay,
            // profiles/r06_event_gap_ab.txt)
            if (sb != st && !onRender) {
                const hipEvent_t shaded = syncEvent(pp, sync++);
                MRT_HIP(hipEventRecord(shaded, st));
                MRT_HIP(hipStreamWaitEvent(sb, shaded, 0));
            }
            if (timing) MRT_HIP(hipEventRecord(poolEvent(pp), ss));
            // the last level (depth > RayDepthMax) shades nothing: no shadow rays
            if (l < nLevels) {
                // the last shadow walk runs alone: a large shard gives it the full grid (C4 N = 1:
                // 13.34 -> 13.29 ms); a small one keeps the narrow grid (N = 8: 2.53 vs 2.55 ms)
                const bool lastAlone = l + 1 == nLevels && r->shadowGridPct == 0 && pathsPerLane >= 8.0;
                launchShadow(r->ds, pp.levels[l], pp.counters, l, onRender ? pp.gstack : pp.gstackShadow, r->gdepth,
                             pp.stats, counting, walkThreads, ss, lastAlone ? 100 : shadowPct);
            }
            if (timing) MRT_HIP(hipEventRecord(poolEvent(pp), ss));
            if (sb != st && !onRender) {
                shadowDone[l] = syncEvent(pp, sync++);
                MRT_HIP(hipEventRecord(shadowDone[l], sb));
            }
        }
        // the resolves wait for every shadow walk on the shadow stream
        const int lastOnShadowStream = lastOnRender ? nLevels - 2 : nLevels;
        if (sb != st && lastOnShadowStream >= 1) MRT_HIP(hipStreamWaitEvent(st, shadowDone[lastOnShadowStream], 0));
        AccumArgs aa{};
        aa.map = map;
        aa.width = r->cfg.width;
        aa.slotBase = slot0;
        aa.nSlots = nChunk;
        aa.spp = spp;
        aa.sampleBase = sampleBase;
        const int topResolve = skipLastShade ? nLevels - 1 : nLevels;
        // level 1's resolve folded into the accumulation (tuning key 34): no level-1 radiance records
        const bool resolveAcc = r->resolveAcc != 0 && topResolve >= 1;
        for (int l = topResolve; l >= (resolveAcc ? 2 : 1); --l) {
            launchResolve(shader, r->ds, pp.levels[l], pp.levels[l + 1], pp.counters, l, sa, r->workGrid, st,
                          skipLastShade && l == nLevels - 1);
        }
        if (!resolveAcc || !launchResolveAccumulate(shader, r->ds, pp.levels[1], pp.levels[2], sa,
                                                    skipLastShade && 1 == nLevels - 1, aa, dBitmap, dPacked, st)) {
            if (resolveAcc)  // (single-level shaders: nothing to resolve)
                launchResolve(shader, r->ds, pp.levels[1], pp.levels[2], pp.counters, 1, sa, r->workGrid, st,
                              skipLastShade && 1 == nLevels - 1);
            launchAccumulate(aa, pp.levels[1].res, dBitmap, dPacked, st);
        }
        // the statistics so far into the pinned host block, the counters reset; after the last chunk
        // the statistics too
        const bool lastChunk = slot0 + nChunk >= r->nSlots;
        launchTally(pp.counters, nLevels, pp.stats, st, skipLast ? nLevels : 0, r->hostStats, lastChunk);
        r->countersClean = true;
        if (lastChunk) r->statsClean = true;
    }
}

// One pass (samples [sampleBase, sampleBase + spp)) with its statistics added to *fs.
// Returns false when the wavefront queues overflowed (the pass's output is then invalid).
bool runPass(mrt_renderer* r, int32_t* dBitmap, int32_t* dPacked, hipStream_t st, int sampleBase, int spp,
             mrt_frame_stats* fs) {
    using namespace mrt;
    const auto t0 = std::chrono::steady_clock::now();
    renderPass(r, dBitmap, dPacked, st, sampleBase, spp);
    MRT_HIP(hipStreamSynchronize(st));  // (k_tally wrote the pass's statistics into r->hostStats)
    unsigned long long hs[kNumStats];
    std::memcpy(hs, r->hostStats, sizeof(hs));
    const auto t1 = std::chrono::steady_clock::now();
    if (hs[kStatOverflow] != 0) return false;
    fs->rays += hs[kStatRays];
    fs->shadowRays += hs[kStatShadowRays];
    fs->walkedRays += hs[kStatRays] - hs[kStatSkipped];
    fs->primaryRays += hs[kStatPrimary];
    fs->nodeRecords += hs[kStatNodes];
    fs->triTests += hs[kStatTris];
    fs->shadowNodeRecords += hs[kStatNodesShadow];
    fs->shadowTriTests += hs[kStatTrisShadow];
    fs->shadowOccluded += hs[kStatOccluded];
    for (int k = 0; k < 16; ++k) fs->walkPhases[k] += hs[kStatPhases + k];
    for (int k = 0; k < 3; ++k) fs->packetWaveRecords[k] += hs[kStatPacket + k];
    fs->leafRecords += hs[kStatLeaves];
    fs->shadowLeafRecords += hs[kStatLeavesShadow];
    for (int l = 0; l < kMaxLevels && l < 16; ++l) {
        fs->levelNodeRecords[l] += hs[kStatLevelNodes + l];
        fs->levelTriTests[l] += hs[kStatLevelTris + l];
        fs->levelLeafRecords[l] += hs[kStatLevelLeaves + l];
        fs->levelShadedVertices[l] += hs[kStatLevelShaded + l];
    }
    fs->maxNodeRecordsPerRay = std::max<uint64_t>(fs->maxNodeRecordsPerRay, hs[kStatMaxNodesRay]);
    fs->shadedVertices += hs[kStatShaded];
    fs->shadeLaunches += r->shadeLaunches;
    for (int l = 0; l < kMaxLevels; ++l) {
        fs->levelRays[l] += hs[kStatLevelRays + l];
        fs->levelShadowRays[l] += hs[kStatLevelShadows + l];
    }
    fs->frameMs += std::chrono::duration<double, std::milli>(t1 - t0).count();
    if (r->profileFlags & 1) {
        const mrt_renderer::Pipe& pp = r->pipe;
        for (size_t e = 0; e + 4 < pp.evCount; e += 5) {
            float ta = 0.0F, tb = 0.0F, tc = 0.0F;
            MRT_HIP(hipEventElapsedTime(&ta, pp.evPool[e], pp.evPool[e + 1]));
            MRT_HIP(hipEventElapsedTime(&tc, pp.evPool[e + 1], pp.evPool[e + 2]));
            MRT_HIP(hipEventElapsedTime(&tb, pp.evPool[e + 3], pp.evPool[e + 4]));
            const size_t lvl = (e / 5) % static_cast<size_t>(r->nLevels);
            if (lvl == 0 && r->fusedL1) {  // one launch: ray generation, walk and shading of level 1
                fs->fusedMs += ta;
                fs->fusedLaunches += 1;
            } else {
                fs->traceMs += ta;
                fs->shadeMs += tc;
            }
            fs->shadowMs += tb;
            fs->levelTraceMs[lvl] += ta;
            fs->levelShadowMs[lvl] += tb;
            const bool last = lvl + 1 == static_cast<size_t>(r->nLevels);
            if (!(r->walkSkipped && last) && !(lvl == 0 && r->fusedL1)) fs->traceLaunches += 1;
            if (!last) fs->shadowLaunches += 1;  // the last level builds no shadow rays
        }
    }
    return true;
}

// a += b for every statistic of a frame (the most node records of one ray: the larger)
void addStats(mrt_frame_stats& a, const mrt_frame_stats& b) {
    using namespace mrt;
    a.rays += b.rays;
    a.shadowRays += b.shadowRays;
    a.walkedRays += b.walkedRays;
    a.primaryRays += b.primaryRays;
    a.nodeRecords += b.nodeRecords;
    a.triTests += b.triTests;
    a.shadowNodeRecords += b.shadowNodeRecords;
    a.shadowTriTests += b.shadowTriTests;
    a.leafRecords += b.leafRecords;
    a.shadowOccluded += b.shadowOccluded;
    for (int k = 0; k < 16; ++k) a.walkPhases[k] += b.walkPhases[k];
    for (int k = 0; k < 3; ++k) a.packetWaveRecords[k] += b.packetWaveRecords[k];
    a.shadowLeafRecords += b.shadowLeafRecords;
    a.fusedMs += b.fusedMs;
    a.fusedLaunches += b.fusedLaunches;
    a.maxNodeRecordsPerRay = std::max(a.maxNodeRecordsPerRay, b.maxNodeRecordsPerRay);
    a.shadedVertices += b.shadedVertices;
    a.shadeLaunches += b.shadeLaunches;
    a.traceMs += b.traceMs;
    a.shadowMs += b.shadowMs;
    a.shadeMs += b.shadeMs;
    a.frameMs += b.frameMs;
    a.traceLaunches += b.traceLaunches;
    a.shadowLaunches += b.shadowLaunches;
    for (int l = 0; l < kMaxLevels && l < 16; ++l) {
        a.levelRays[l] += b.levelRays[l];
        a.levelShadowRays[l] += b.levelShadowRays[l];
        a.levelTraceMs[l] += b.levelTraceMs[l];
        a.levelShadowMs[l] += b.levelShadowMs[l];
        a.levelNodeRecords[l] += b.levelNodeRecords[l];
        a.levelTriTests[l] += b.levelTriTests[l];
        a.levelLeafRecords[l] += b.levelLeafRecords[l];
        a.levelShadedVertices[l] += b.levelShadedVertices[l];
    }
}

// Progressive mode: sample smp's pass, its statistics added to *fs.  The running average is read
// by the pass: a copy is kept to redo a pass whose queues overflowed (in smaller chunks).
void renderProgressiveSample(mrt_renderer* r, int32_t* dBitmap, int32_t* dPacked, hipStream_t st, int smp,
                             mrt_frame_stats* fs) {
    const size_t npx = static_cast<size_t>(r->cfg.width) * static_cast<size_t>(r->cfg.height);
    int32_t* acc = dBitmap != nullptr ? dBitmap : dPacked;
    const size_t accN = dBitmap != nullptr ? npx : static_cast<size_t>(r->nSlots);
    if (r->dBackup == nullptr || r->backupN < accN) {
        r->dBackup = r->frameMem.alloc<int32_t>(accN);
        r->backupN = accN;
    }
    for (int attempt = 0; attempt < 4; ++attempt) {
        if (acc != nullptr) MRT_HIP(hipMemcpyAsync(r->dBackup, acc, accN * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
        mrt_frame_stats pass{};
        if (runPass(r, dBitmap, dPacked, st, smp, 1, &pass)) {
            addStats(*fs, pass);
            return;
        }
        if (acc != nullptr) MRT_HIP(hipMemcpyAsync(acc, r->dBackup, accN * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
        allocQueues(r, std::max(1, r->chunkSlots / 2), 2);
    }
    throw std::runtime_error("wavefront queue overflow persists after shrinking the chunk");
}

// Renderer::renderFrame (Renderer.cpp:53-88): samples 0..spp-1 averaged with incrementalAvg.
// Default: every sample of the frame in flight at once (one wavefront pass per chunk).
// cfg.progressive: one pass per sample, the bitmap (and hostBitmap, if given) updated and
// getSample() advanced after each, stopRender() honoured between samples - the reference's
// progressive contract for the Qt / Android front ends.  Both give the same final bitmap.
// One renderer (one GPU, or one shard of a device group).
void renderFrameSingle(mrt_renderer* r, int32_t* dBitmap, int32_t* dPacked, hipStream_t st,
                       int32_t* hostBitmap = nullptr) {
    using namespace mrt;
    // (a device group's head is its shard 0 too: the group keeps getSample() itself)
    const bool groupHead = !r->peers.empty();
    if (!groupHead) r->sample.store(0);
    if (r->stopFlag.load()) return;  // stopRender zeroes samplesPixel_ (Renderer.cpp:97)
    const int spp = std::max(1, r->cfg.samplesPixel);
    const size_t npx = static_cast<size_t>(r->cfg.width) * static_cast<size_t>(r->cfg.height);
    mrt_frame_stats fs{};
    if (r->cfg.progressive == 0) {
        bool done = false;
        for (int attempt = 0; attempt < 4 && !done; ++attempt) {
            fs = mrt_frame_stats{};
            done = runPass(r, dBitmap, dPacked, st, 0, spp, &fs);
            if (!done) allocQueues(r, std::max(1, r->chunkSlots / 2), 2);  // same results, more passes
        }
        if (!done) throw std::runtime_error("wavefront queue overflow persists after shrinking the chunk");
        if (hostBitmap != nullptr && dBitmap != nullptr) {
            MRT_HIP(hipMemcpyAsync(hostBitmap, dBitmap, npx * sizeof(int32_t), hipMemcpyDeviceToHost, st));
            MRT_HIP(hipStreamSynchronize(st));
        }
        if (!r->stopFlag.load() && !groupHead) r->sample.store(r->cfg.samplesPixel);
    } else {
        for (int smp = 0; smp < spp && !r->stopFlag.load(); ++smp) {
            renderProgressiveSample(r, dBitmap, dPacked, st, smp, &fs);
            if (hostBitmap != nullptr && dBitmap != nullptr) {
                MRT_HIP(hipMemcpyAsync(hostBitmap, dBitmap, npx * sizeof(int32_t), hipMemcpyDeviceToHost, st));
                MRT_HIP(hipStreamSynchronize(st));
            }
            if (!groupHead) r->sample.store(smp + 1);  // Renderer.cpp:82-86
        }
    }
    r->last = fs;
    r->totalRays.fetch_add(fs.rays + fs.shadowRays);
}

// The frame's assembly from rankCount packed shards (d_gathered: rankCount slices of maxSlots
// entries): one k_unpack_ranks launch per kUnpackRanks shards (a launch per shard cost ~8 us each
// at N = 8).
void unpackGathered(const mrt_renderer* r, const int32_t* dGathered, int32_t* dBitmap, hipStream_t st) {
    for (int k0 = 0; k0 < r->rankCount; k0 += mrt::kUnpackRanks) {
        mrt::UnpackArgs a{};
        a.width = r->cfg.width;
        a.first = k0;
        a.stride = r->maxSlots;
        const int ranks = std::min(mrt::kUnpackRanks, r->rankCount - k0);
        int maxN = 0;
        for (int j = 0; j < ranks; ++j) {
            const auto k = static_cast<size_t>(k0 + j);
            const auto& pre = r->prefixByRank[k];
            const auto& un = r->unitsByRank[k];
            a.maps[j] = r->mapByRank[k];
            a.n[j] = un.empty() ? 0 : pre.back() + un.back().z * un.back().w;
            maxN = std::max(maxN, a.n[j]);
        }
        mrt::launchUnpackRanks(a, ranks, maxN, dGathered, dBitmap, st);
    }
}

// ---- device groups (mrt_config.devices) ------------------------------------------------------
// Renderer::renderFrame hands the frame's tiles to its worker threads (Renderer.cpp:62-82); a
// device group hands its screen-tile shards to its GPUs, one host thread per shard.

mrt_renderer* shardOf(mrt_renderer* r, int i) { return i == 0 ? r : r->peers[static_cast<size_t>(i - 1)].get(); }
int groupSize(const mrt_renderer* r) { return 1 + static_cast<int>(r->peers.size()); }

// f(shard, i) for every shard of the group, shard i on the head's shard worker i (bound to its
// device; shard 0 in the calling thread); the first failure is rethrown after all have finished
template <class F>
void forEachShard(mrt_renderer* r, F&& f) {
    MRT_HIP(hipSetDevice(r->device));
    r->shardPool->run([&](int i) { f(shardOf(r, i), i); });
}

// The shards' packed pixels into the head's gather buffer (peer copies over xGMI; a shard on the
// head's own GPU: a device-to-device copy), then the frame from them, on the head's stream st.
// Every shard's render has completed (its passes end with a stream synchronisation).
void assembleGroup(mrt_renderer* r, int32_t* dBitmap, hipStream_t st) {
    if (dBitmap == nullptr) return;
    for (int i = 0; i < groupSize(r); ++i) {
        const mrt_renderer* p = shardOf(r, i);
        int32_t* dst = r->dGathered + static_cast<size_t>(i) * static_cast<size_t>(r->maxSlots);
        const size_t bytes = sizeof(int32_t) * static_cast<size_t>(p->nSlots);
        if (bytes == 0) continue;
        if (p->device == r->device)
            MRT_HIP(hipMemcpyAsync(dst, p->dOwnPacked, bytes, hipMemcpyDeviceToDevice, st));
        else
            MRT_HIP(hipMemcpyPeerAsync(dst, r->device, p->dOwnPacked, p->device, bytes, st));
    }
    unpackGathered(r, r->dGathered, dBitmap, st);
}

// One frame of a device group into dBitmap (on the head's device; may be null) and, if given, the
// host bitmap.  getSample() and stopRender() keep their meaning for the whole group: the sample
// count advances once every shard has it, a stop reaches every shard (mrt_stop_render).
void renderGroupFrame(mrt_renderer* r, int32_t* dBitmap, hipStream_t st, int32_t* hostBitmap) {
    r->sample.store(0);
    if (r->stopFlag.load()) return;
    const auto t0 = std::chrono::steady_clock::now();
    const int n = groupSize(r);
    const int spp = std::max(1, r->cfg.samplesPixel);
    const size_t npx = static_cast<size_t>(r->cfg.width) * static_cast<size_t>(r->cfg.height);
    const uint64_t rays0 = r->totalRays.load();
    std::vector<mrt_frame_stats> shardStats(static_cast<size_t>(n));
    auto toHost = [&] {
        if (hostBitmap == nullptr || dBitmap == nullptr) return;
        MRT_HIP(hipMemcpyAsync(hostBitmap, dBitmap, npx * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        MRT_HIP(hipStreamSynchronize(st));
    };
    if (r->cfg.progressive == 0) {
        forEachShard(r, [&](mrt_renderer* p, int i) {
            renderFrameSingle(p, nullptr, p->dOwnPacked, p->stream);
            shardStats[static_cast<size_t>(i)] = p->last;
        });
        assembleGroup(r, dBitmap, st);
        toHost();
        if (!r->stopFlag.load()) r->sample.store(r->cfg.samplesPixel);
    } else {
        for (int smp = 0; smp < spp && !r->stopFlag.load(); ++smp) {
            forEachShard(r, [&](mrt_renderer* p, int i) {
                renderProgressiveSample(p, nullptr, p->dOwnPacked, p->stream, smp, &shardStats[static_cast<size_t>(i)]);
            });
            assembleGroup(r, dBitmap, st);
            toHost();
            r->sample.store(smp + 1);  // Renderer.cpp:82-86
        }
        for (int i = 1; i < n; ++i) shardOf(r, i)->last = shardStats[static_cast<size_t>(i)];
    }
    mrt_frame_stats fs{};
    for (const mrt_frame_stats& x : shardStats) addStats(fs, x);
    // the group's frame time is its wall time (the shards run at the same time), not the shards' sum:
    // until every shard has finished and the assembly is queued; the per-kernel durations stay summed
    // over the shards (mrt_frame_stats)
    fs.frameMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    r->last = fs;
    r->totalRays.store(rays0 + fs.rays + fs.shadowRays);
}

void renderFrameDevice(mrt_renderer* r, int32_t* dBitmap, int32_t* dPacked, hipStream_t st,
                       int32_t* hostBitmap = nullptr) {
    if (r->peers.empty()) {
        renderFrameSingle(r, dBitmap, dPacked, st, hostBitmap);
        return;
    }
    if (dPacked != nullptr) throw std::runtime_error("a device group assembles its frame itself: no packed output");
    renderGroupFrame(r, dBitmap, st, hostBitmap);
}

void stopAll(mrt_renderer* r) {
    r->stopFlag.store(true);
    for (auto& p : r->peers) p->stopFlag.store(true);
}

// An OBJ scene handed over as text (the Android front end reads the files through descriptors,
// JNI_layer.cpp:994-1063) with its map_Kd textures by file name.
struct MemScene {
    std::string obj, mtl, cam;
    std::map<std::string, std::string> textures;
};

mrt_renderer* createGroup(const mrt_config* cfg, const MemScene* mem);

mrt_renderer* createRenderer(const mrt_config* cfg, const MemScene* mem = nullptr) {
    using namespace mrt;
    if (cfg->deviceCount > 1) return createGroup(cfg, mem);
    auto r = std::make_unique<mrt_renderer>();
    r->keepHost = mem != nullptr;
    r->cfg = *cfg;
    r->objPath = cfg->objFilePath ? cfg->objFilePath : "";
    r->mtlPath = cfg->mtlFilePath ? cfg->mtlFilePath : "";
    r->camPath = cfg->camFilePath ? cfg->camFilePath : "";
    r->cfg.objFilePath = r->objPath.c_str();
    r->cfg.mtlFilePath = r->mtlPath.c_str();
    r->cfg.camFilePath = r->camPath.c_str();
    r->maxDepth = cfg->maxDepth > 0 ? cfg->maxDepth : kRayDepthMaxDefault;
    if (r->maxDepth + 2 >= kMaxLevels) throw std::runtime_error("maxDepth too large");
    r->rankCount = cfg->rankCount > 0 ? cfg->rankCount : 1;
    r->rankIndex = cfg->rankIndex;
    if (r->rankIndex < 0 || r->rankIndex >= r->rankCount) throw std::runtime_error("rankIndex out of range");
    // C_wrapper.cpp:153-193: 1 Whitted, 2 PathTracer, 3 DepthMap, 4 DiffuseMaterial, else NoShadows
    r->shader = (cfg->shader >= kShaderWhitted && cfg->shader <= kShaderDiffuse) ? cfg->shader : kShaderNoShadows;
    r->nLevels = (r->shader == kShaderWhitted || r->shader == kShaderPathTracer) ? r->maxDepth + 1 : 1;
    if (cfg->width < 16 || cfg->height < 16) throw std::runtime_error("width/height must be >= 16");
    if (cfg->samplesPixel < 1 || cfg->samplesLight < 1) throw std::runtime_error("samplesPixel/samplesLight must be >= 1");
    if (cfg->device >= 0) MRT_HIP(hipSetDevice(cfg->device));
    MRT_HIP(hipGetDevice(&r->device));
    MRT_HIP(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
    MRT_HIP(hipEventCreateWithFlags(&r->joinIn, hipEventDisableTiming));
    MRT_HIP(hipEventCreateWithFlags(&r->joinOut, hipEventDisableTiming));
    hipDeviceProp_t prop;
    MRT_HIP(hipGetDeviceProperties(&prop, r->device));
    r->traceThreads = prop.multiProcessorCount * traceResidentThreadsPerCU();
    r->workGrid = prop.multiProcessorCount * 8;
    r->cus = prop.multiProcessorCount;

    // scene (C_wrapper.cpp:68-141)
    const float ratio = static_cast<float>(cfg->width) / static_cast<float>(cfg->height);
    HScene sc;
    r->maxPoint = v3{1.0F, 1.0F, 1.0F};
    if (cfg->sceneIndex >= 0 && cfg->sceneIndex <= 3) {
        sc = builtinScene(cfg->sceneIndex);
        r->cam = builtinCamera(cfg->sceneIndex, ratio);
        r->maxPoint = builtinMaxPoint(cfg->sceneIndex);
    } else if (mem != nullptr) {
        if (mem->obj.empty()) throw std::runtime_error("OBJ file not read!");  // JNI_layer.cpp:552-555
        std::string err;
        std::istringstream obj(mem->obj), mtl(mem->mtl), cam(mem->cam);
        const TextureSource textures = [mem](const std::string& name, HTexture* tex) {
            const auto it = mem->textures.find(name.substr(name.find_last_of('/') + 1));
            if (it == mem->textures.end()) return false;
            std::string terr;
            return decodePng(std::vector<uint8_t>(it->second.begin(), it->second.end()), tex, &terr);
        };
        if (!loadObjStreams(obj, mem->mtl.empty() ? nullptr : &mtl, textures, &sc, &err)) throw std::runtime_error(err);
        if (!loadCameraStream(cam, ratio, &r->cam, &err, "camera definition")) throw std::runtime_error(err);
    } else {
        std::string err;
        if (!loadObjScene(r->objPath, r->mtlPath, &sc, &err)) throw std::runtime_error(err);
        if (!loadCameraFile(r->camPath, ratio, &r->cam, &err)) throw std::runtime_error(err);
    }
    uploadScene(r.get(), sc);
    createShadowStream(r.get());
    buildUnits(r.get());
    allocQueues(r.get(), chunkFor(r.get()), 2);
    const size_t npx = static_cast<size_t>(r->cfg.width) * static_cast<size_t>(r->cfg.height);
    r->dBitmap = r->frameMem.alloc<int32_t>(npx);
    MRT_HIP(hipMemsetAsync(r->dBitmap, 0, sizeof(int32_t) * npx, r->stream));
    MRT_HIP(hipStreamSynchronize(r->stream));
    return r.release();
}

// A device group (mrt_config.devices): one renderer per shard, created concurrently (each parses
// and uploads the scene on its own GPU), shard 0 the head.  The head enables peer access to the
// other GPUs where the platform allows it (xGMI); hipMemcpyPeerAsync works either way.
mrt_renderer* createGroup(const mrt_config* cfg, const MemScene* mem) {
    const int n = cfg->deviceCount;
    if (cfg->devices == nullptr) throw std::runtime_error("deviceCount > 1 needs the devices array");
    if (cfg->rankCount > 1 || cfg->rankIndex != 0)
        throw std::runtime_error("a device group shards the frame itself: leave rankIndex / rankCount at 0 / 1");
    int visible = 0;
    MRT_HIP(hipGetDeviceCount(&visible));
    for (int i = 0; i < n; ++i)
        if (cfg->devices[i] < 0 || cfg->devices[i] >= visible)
            throw std::runtime_error("device group: ordinal " + std::to_string(cfg->devices[i]) + " not among the " +
                                     std::to_string(visible) + " visible GPUs");
    std::vector<std::unique_ptr<mrt_renderer>> shards(static_cast<size_t>(n));
    std::vector<std::exception_ptr> err(static_cast<size_t>(n));
    std::vector<std::thread> th;
    for (int i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            try {
                mrt_config c = *cfg;
                c.devices = nullptr;
                c.deviceCount = 0;
                c.device = cfg->devices[i];
                c.rankIndex = i;
                c.rankCount = n;
                shards[static_cast<size_t>(i)].reset(createRenderer(&c, mem));
                mrt_renderer* p = shards[static_cast<size_t>(i)].get();
                p->dOwnPacked = p->frameMem.alloc<int32_t>(static_cast<size_t>(std::max(1, p->nSlots)));
            } catch (...) {
                err[static_cast<size_t>(i)] = std::current_exception();
            }
        });
    for (std::thread& t : th) t.join();
    for (const std::exception_ptr& e : err)
        if (e) std::rethrow_exception(e);
    std::unique_ptr<mrt_renderer> head = std::move(shards[0]);
    MRT_HIP(hipSetDevice(head->device));
    head->dGathered = head->frameMem.alloc<int32_t>(static_cast<size_t>(n) * static_cast<size_t>(std::max(1, head->maxSlots)));
    for (int i = 1; i < n; ++i) {
        const int d = cfg->devices[i];
        int can = 0;
        if (d != head->device && hipDeviceCanAccessPeer(&can, head->device, d) == hipSuccess && can) {
            const hipError_t e = hipDeviceEnablePeerAccess(d, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) MRT_HIP(e);
            (void)hipGetLastError();
        }
        head->peers.push_back(std::move(shards[static_cast<size_t>(i)]));
    }
    head->shardPool = std::make_unique<ShardPool>(std::vector<int>(cfg->devices, cfg->devices + n));
    return head.release();
}

template <class F>
int guarded(F&& f) {
    try {
        f();
        return 0;
    } catch (const std::exception& e) {
        gLastError = e.what();
    } catch (...) {
        gLastError = "unknown error";
    }
    return -1;
}

}  // namespace

extern "C" {

const char* mrt_last_error(void) { return gLastError.c_str(); }

int mrt_create(const mrt_config* cfg, mrt_renderer** out) {
    *out = nullptr;
    return guarded([&] { *out = createRenderer(cfg); });
}

int mrt_create_from_memory(const mrt_config* cfg, const char* obj, int64_t objLen, const char* mtl, int64_t mtlLen,
                           const char* cam, int64_t camLen, const mrt_blob* textures, int32_t nTextures,
                           mrt_renderer** out) {
    *out = nullptr;
    return guarded([&] {
        MemScene m;
        if (obj != nullptr && objLen > 0) m.obj.assign(obj, static_cast<size_t>(objLen));
        if (mtl != nullptr && mtlLen > 0) m.mtl.assign(mtl, static_cast<size_t>(mtlLen));
        if (cam != nullptr && camLen > 0) m.cam.assign(cam, static_cast<size_t>(camLen));
        for (int32_t i = 0; i < nTextures; ++i) {
            const mrt_blob& b = textures[i];
            m.textures[b.name != nullptr ? b.name : ""].assign(reinterpret_cast<const char*>(b.bytes),
                                                                static_cast<size_t>(b.size));
        }
        *out = createRenderer(cfg, &m);
    });
}

int64_t mrt_preview_arrays(const mrt_renderer* r, float* vertices, float* colors, float* camera) {
    using namespace mrt;
    if (!r->keepHost) {
        gLastError = "preview arrays: the renderer keeps no host scene (create it with mrt_create_from_memory)";
        return -1;
    }
    size_t i = 0, j = 0;
    for (const HTriangle& t : r->hostTris) {
        // rtInitVerticesArray (JNI_layer.cpp:243-311): A, A + AB, A + AC with z negated for GL
        const v3 a = t.A, b = v3{a.x + t.AB.x, a.y + t.AB.y, a.z + t.AB.z}, c = v3{a.x + t.AC.x, a.y + t.AC.y, a.z + t.AC.z};
        if (vertices != nullptr)
            for (const v3& p : {a, b, c}) {
                vertices[i++] = p.x;
                vertices[i++] = p.y;
                vertices[i++] = -p.z;
                vertices[i++] = 1.0F;
            }
        // rtInitColorsArray (:314-389): Kd, replaced by Ks / Kt / Le where each is greater in all
        // three components
        if (colors != nullptr) {
            HMaterial m;
            if (t.mat >= 0) m = r->hostMats[static_cast<size_t>(t.mat)];
            auto greater = [](v3 x, v3 y) { return x.x > y.x && x.y > y.y && x.z > y.z; };
            v3 col = m.Kd;
            col = greater(m.Ks, col) ? m.Ks : col;
            col = greater(m.Kt, col) ? m.Kt : col;
            col = greater(m.Le, col) ? m.Le : col;
            for (int k = 0; k < 3; ++k) {
                colors[j++] = col.x;
                colors[j++] = col.y;
                colors[j++] = col.z;
                colors[j++] = 1.0F;
            }
        }
    }
    if (camera != nullptr) {  // rtInitCameraArray (:153-240)
        const GCamera& c = r->cam;
        const v3 rows[4] = {c.position, c.direction, c.up, c.right};
        for (int k = 0; k < 4; ++k) {
            camera[4 * k] = rows[k].x;
            camera[4 * k + 1] = rows[k].y;
            camera[4 * k + 2] = rows[k].z;
            camera[4 * k + 3] = 1.0F;
        }
        if (c.kind == 0) {  // Perspective::getHFov / getVFov in degrees (Camera.cpp:50-53)
            camera[16] = (c.hFov / kPi) * 180.0F;
            camera[17] = (c.vFov / kPi) * 180.0F;
            camera[18] = 0.0F;
            camera[19] = 0.0F;
        } else {  // Orthographic::getSizeH / getSizeV (the half sizes)
            camera[16] = 0.0F;
            camera[17] = 0.0F;
            camera[18] = c.hFov;
            camera[19] = c.vFov;
        }
    }
    return static_cast<int64_t>(r->hostTris.size());
}

void mrt_destroy(mrt_renderer* r) {
    if (r != nullptr) {
        (void)hipStreamSynchronize(r->stream);
        for (auto& p : r->peers) (void)hipStreamSynchronize(p->stream);
        delete r;
    }
}

int mrt_render_frame(mrt_renderer* r, int32_t* bitmap) {
    return guarded([&] {
        MRT_HIP(hipSetDevice(r->device));  // the calling thread may not be the one that created r
        const size_t n = static_cast<size_t>(r->cfg.width) * static_cast<size_t>(r->cfg.height);
        MRT_HIP(hipMemcpyAsync(r->dBitmap, bitmap, n * sizeof(int32_t), hipMemcpyHostToDevice, r->stream));
        renderFrameDevice(r, r->dBitmap, nullptr, r->stream, bitmap);
    });
}

int mrt_render_frame_device(mrt_renderer* r, int32_t* dBitmap, int32_t* dPacked, void* stream) {
    return guarded([&] {
        MRT_HIP(hipSetDevice(r->device));
        hipStream_t st = stream != nullptr ? static_cast<hipStream_t>(stream) : r->stream;
        if (st == r->stream) {
            renderFrameDevice(r, dBitmap, dPacked, st);
            return;
        }
        // the frame on the renderer's stream (its hardware queue is known to differ from the shadow
        // stream's), ordered after the caller's work and before the caller's next.  (A single
        // renderer's frame ends with its stream synchronised - runPass reads the pass's statistics -
        // so only a device group's assembly, queued after its shards, needs the second event.)
        MRT_HIP(hipEventRecord(r->joinIn, st));
        MRT_HIP(hipStreamWaitEvent(r->stream, r->joinIn, 0));
        renderFrameDevice(r, dBitmap, dPacked, r->stream);
        if (!r->peers.empty()) {
            MRT_HIP(hipEventRecord(r->joinOut, r->stream));
            MRT_HIP(hipStreamWaitEvent(st, r->joinOut, 0));
        }
    });
}

int mrt_unpack_gathered(mrt_renderer* r, const int32_t* dGathered, int32_t* dBitmap, void* stream) {
    return guarded([&] {
        hipStream_t st = stream != nullptr ? static_cast<hipStream_t>(stream) : r->stream;
        unpackGathered(r, dGathered, dBitmap, st);
    });
}

int mrt_stop_render(mrt_renderer* r) {
    stopAll(r);
    return 0;
}

int32_t mrt_get_sample(const mrt_renderer* r) { return r->sample.load(); }

uint64_t mrt_get_total_casted_rays(const mrt_renderer* r) { return r->totalRays.load(); }

int mrt_get_scene_info(const mrt_renderer* r, mrt_scene_info* info) {
    info->triangles = r->nTri;
    info->lights = r->nLights;
    info->planes = r->nPlanes;
    info->spheres = r->nSpheres;
    info->materials = r->nMats;
    info->triangleNodes = r->nTriNodes;
    info->triangleBvhDepth = r->triDepth;
    info->pixelSlots = r->nSlots;
    info->pixelSlotsMax = r->maxSlots;
    info->deviceBytes = static_cast<int64_t>(r->sceneMem.total + r->queueMem.total + r->frameMem.total);
    info->shadowStreamConcurrent = r->shadowConcurrent;
    info->shadowStreamsTried = r->shadowTries;
    info->deviceCount = groupSize(r);
    for (const auto& p : r->peers) {  // a device group: the whole frame's slots, every GPU's memory
        info->pixelSlots += p->nSlots;
        info->deviceBytes += static_cast<int64_t>(p->sceneMem.total + p->queueMem.total + p->frameMem.total);
        info->shadowStreamConcurrent = std::min<int64_t>(info->shadowStreamConcurrent, p->shadowConcurrent);
    }
    return 0;
}

int mrt_set_camera(mrt_renderer* r, int32_t kind, const float* position, const float* lookAt, const float* up,
                   float a, float b) {
    return guarded([&] {
        if (r == nullptr || position == nullptr || lookAt == nullptr || up == nullptr)
            throw std::runtime_error("mrt_set_camera: null argument");
        if (!std::isfinite(a) || !std::isfinite(b)) throw std::runtime_error("mrt_set_camera: non-finite field of view / size");
        for (int k = 0; k < 3; ++k)
            if (!std::isfinite(position[k]) || !std::isfinite(lookAt[k]) || !std::isfinite(up[k]))
                throw std::runtime_error("mrt_set_camera: non-finite position / lookAt / up");
        const mrt::v3 p{position[0], position[1], position[2]}, l{lookAt[0], lookAt[1], lookAt[2]},
            u{up[0], up[1], up[2]};
        mrt::GCamera cam;
        if (kind == 0) {
            cam = mrt::makePerspective(p, l, u, a, b);
        } else if (kind == 1) {
            cam = mrt::makeOrthographic(p, l, u, a, b);
        } else {
            throw std::runtime_error("camera kind: 0 perspective, 1 orthographic");
        }
        for (int i = 0; i < groupSize(r); ++i) shardOf(r, i)->cam = cam;
    });
}

int mrt_set_pixel_sampler(mrt_renderer* r, int32_t kind, float value) {
    if (r == nullptr) {
        gLastError = "mrt_set_pixel_sampler: null renderer";
        return -1;
    }
    if (kind < -1 || kind > 1) {
        gLastError = "pixel sampler: -1 by samplesPixel, 0 Constant, 1 StaticHaltonSeq";
        return -1;
    }
    for (int i = 0; i < groupSize(r); ++i) {
        shardOf(r, i)->pixelSampler = kind;
        shardOf(r, i)->pixelConst = value;
    }
    return 0;
}

int mrt_set_max_point(mrt_renderer* r, const float* maxPoint) {
    return guarded([&] {
        if (r == nullptr || maxPoint == nullptr) throw std::runtime_error("mrt_set_max_point: null argument");
        for (int i = 0; i < groupSize(r); ++i) shardOf(r, i)->maxPoint = mrt::v3{maxPoint[0], maxPoint[1], maxPoint[2]};
    });
}

int mrt_set_profiling(mrt_renderer* r, int32_t flags) {
    for (int i = 0; i < groupSize(r); ++i) shardOf(r, i)->profileFlags = flags;
    return 0;
}

int64_t mrt_wave_log(mrt_renderer* r, uint64_t* out) {
    using namespace mrt;
    if (r == nullptr) return -1;
    if (out == nullptr) return kWaveLogEntries;
    int64_t n = -1;
    const int rc = guarded([&] {
        if (r->pipe.stats == nullptr) throw std::runtime_error("no frame rendered");
        MRT_HIP(hipSetDevice(r->device));
        MRT_HIP(hipMemcpy(out, r->pipe.stats + kNumStats, sizeof(uint64_t) * kWaveLogEntries, hipMemcpyDeviceToHost));
        n = kWaveLogEntries;
    });
    return rc == 0 ? n : -1;
}

static int setTuningOne(mrt_renderer* r, int32_t key, int32_t value);

int mrt_set_tuning(mrt_renderer* r, int32_t key, int32_t value) {
    for (int i = 0; i < groupSize(r); ++i) {  // every shard of a device group alike
        const int rc = setTuningOne(shardOf(r, i), key, value);
        if (rc != 0) return rc;
    }
    return 0;
}

static int setTuningOne(mrt_renderer* r, int32_t key, int32_t value) {
    if (key == 1 && value >= 0 && value < mrt::kTraceVariants) {
        r->ds.variant = value;
        return 0;
    }
    if (key == 2 && value >= 0 && value <= 3) {
        r->ds.cull = value;
        return 0;
    }
    if (key == 3 && (value == 0 || value == 1)) {
        r->overlap = value;
        return 0;
    }
    if (key == 7 && (value == 0 || value == 1)) {
        r->skipLast = value;
        return 0;
    }
    if (key == 5 && (value == 0 || value == 1)) {
        r->ds.anyOrder = value;
        return 0;
    }
    if (key == 11 && value >= -1 && value <= 64) {
        r->shadeGridPerCU = value;
        return 0;
    }
    if (key == 10 && (value == 0 || value == 1)) {
        r->ds.leanShade = value;
        return 0;
    }
    if (key == 9 && value >= 0 && value <= 64) {
        r->refill = value;
        return 0;
    }
    if (key == 8 && (value == 0 || value == 1)) {
        r->ds.tailDonate = value;
        return 0;
    }
    if (key == 16 && (value == 0 || value == 1)) {
        if (value == 1 && r->stackNeed > mrt::kPacketStack) {
            gLastError = "packet walk: the walk tree needs a deeper stack";
            return -1;
        }
        r->ds.packet = value;
        return 0;
    }
    if (key == 17 && value >= -1 && value <= 1) {
        r->fuseL1Mode = value;
        return 0;
    }
    if (key == 27 && (value == 0 || value == 1)) {
        r->lastShadowRender = value;
        return 0;
    }
    if (key == 33 && value >= 0 && value <= 2) {
        r->genL1 = value;
        return 0;
    }
    if (key == 34 && (value == 0 || value == 1)) {
        r->resolveAcc = value;
        return 0;
    }
    if (key == 35 && (value == 0 || value == 1)) {
        r->shadeWaitsShadow = value;
        return 0;
    }

    if (key == 28 && value >= 0 && value <= 65536) {
        r->walkGridCap = value;
        return 0;
    }
    if (key == 6 && value >= 0 && value <= 100) {
        r->shadowGridPct = value;
        return 0;
    }
    gLastError = "unknown tuning key/value";
    return -1;
}

int64_t mrt_triangle_bvh(const mrt_config* cfg, float* boxes, int32_t* offsets, int32_t* counts, int32_t* order) {
    using namespace mrt;
    int64_t n = -1;
    const int rc = guarded([&] {
        HScene sc;
        if (cfg->sceneIndex >= 0 && cfg->sceneIndex <= 3) {
            sc = builtinScene(cfg->sceneIndex);
        } else {
            std::string err;
            if (!loadObjScene(cfg->objFilePath ? cfg->objFilePath : "", cfg->mtlFilePath ? cfg->mtlFilePath : "", &sc,
                              &err))
                throw std::runtime_error(err);
        }
        std::vector<int32_t> perm;
        const std::vector<HBVHNode> nodes = buildBVH(&sc.triangles, &perm);
        n = static_cast<int64_t>(nodes.size());
        if (boxes == nullptr) return;
        for (size_t i = 0; i < nodes.size(); ++i) {
            const HBVHNode& b = nodes[i];
            const float v[6] = {b.box.mn.x, b.box.mn.y, b.box.mn.z, b.box.mx.x, b.box.mx.y, b.box.mx.z};
            std::memcpy(boxes + 6 * i, v, sizeof(v));
            offsets[i] = b.indexOffset;
            counts[i] = b.numPrimitives;
        }
        std::memcpy(order, perm.data(), perm.size() * sizeof(int32_t));
    });
    return rc == 0 ? n : -1;
}

int64_t mrt_walk_tree(const mrt_config* cfg, uint32_t* nodes, float* grid, int32_t* root) {
    using namespace mrt;
    int64_t n = -1;
    const int rc = guarded([&] {
        HScene sc;
        // the camera too: the collapse weighs nodes by the frame's rays, as the renderer does
        const float ratio = cfg->height > 0 ? static_cast<float>(cfg->width) / static_cast<float>(cfg->height) : 1.0F;
        GCamera cam{};
        bool haveCam = true;
        if (cfg->sceneIndex >= 0 && cfg->sceneIndex <= 3) {
            sc = builtinScene(cfg->sceneIndex);
            cam = builtinCamera(cfg->sceneIndex, ratio);
        } else {
            std::string err;
            if (!loadObjScene(cfg->objFilePath ? cfg->objFilePath : "", cfg->mtlFilePath ? cfg->mtlFilePath : "", &sc,
                              &err))
                throw std::runtime_error(err);
            haveCam = loadCameraFile(cfg->camFilePath ? cfg->camFilePath : "", ratio, &cam, &err);
        }
        std::vector<int32_t> perm;
        const std::vector<HBVHNode> tn = buildBVH(&sc.triangles, &perm);
        GRoot r{};
        QGrid g{};
        std::vector<QNode4> qn;
        int top = 0;
        const int maxDepth = cfg->maxDepth > 0 ? cfg->maxDepth : kRayDepthMaxDefault;
        std::vector<double> cost;
        const std::vector<HBVHNode> wn = haveCam ? frameWalkTree(walkTreeOver(tn), sc, cam, cfg->width, cfg->height, maxDepth, &cost)
                                                 : walkTreeOver(tn);
        if (!toQuantizedBVH4(wn, sc.triangles.size(), &r, kTopNodesMax, &top, &g, &qn, nullptr,
                             cost.empty() ? nullptr : &cost))
            throw std::runtime_error("walk tree not quantizable (non-finite boxes)");
        n = static_cast<int64_t>(qn.size());
        if (nodes != nullptr) std::memcpy(nodes, qn.data(), qn.size() * sizeof(QNode4));
        if (grid != nullptr) {
            std::memcpy(grid, g.origin, sizeof(g.origin));
            std::memcpy(grid + 3, g.step, sizeof(g.step));
        }
        if (root != nullptr) {
            root[0] = r.ref;
            root[1] = r.count;
            root[2] = kWalkWidth;
        }
    });
    return rc == 0 ? n : -1;
}

int mrt_grid_box_test(int32_t kind, const float* prim, const float* box) {
    using namespace mrt;
    const HAABB b{v3{box[0], box[1], box[2]}, v3{box[3], box[4], box[5]}};
    const v3 p0{prim[0], prim[1], prim[2]}, p1{prim[3], prim[4], prim[5]};
    if (kind == 0) return boxIntersect(makeTriangle(p0, p1, v3{prim[6], prim[7], prim[8]}), b) ? 1 : 0;
    if (kind == 1) return boxIntersect(makePlane(p0, p1, -1), b) ? 1 : 0;
    if (kind == 2) return boxIntersect(makeSphere(p0, prim[3], -1), b) ? 1 : 0;
    gLastError = "grid box test: kind must be 0 (triangle), 1 (plane) or 2 (sphere)";
    return -1;
}

int64_t mrt_regular_grid(const mrt_config* cfg, int32_t kind, float* world, int32_t* start, int32_t* items) {
    using namespace mrt;
    int64_t n = -1;
    const int rc = guarded([&] {
        if (kind < 0 || kind > 2) throw std::runtime_error("regular grid: kind must be 0 (planes), 1 (spheres), 2 (triangles)");
        HScene sc;
        if (cfg->sceneIndex >= 0 && cfg->sceneIndex <= 3) {
            sc = builtinScene(cfg->sceneIndex);
        } else {
            std::string err;
            if (!loadObjScene(cfg->objFilePath ? cfg->objFilePath : "", cfg->mtlFilePath ? cfg->mtlFilePath : "", &sc,
                              &err))
                throw std::runtime_error(err);
        }
        std::vector<int32_t> order;
        HGrid g;
        if (kind == 0) {
            buildBVH(&sc.planes, &order);
            g = buildGrid(sc.planes, order);
        } else if (kind == 1) {
            buildBVH(&sc.spheres, &order);
            g = buildGrid(sc.spheres, order);
        } else {
            buildBVH(&sc.triangles, &order);
            g = buildGrid(sc.triangles, order);
        }
        n = static_cast<int64_t>(g.items.size());
        if (world != nullptr) {
            const float w[12] = {g.world.mn.x, g.world.mn.y, g.world.mn.z, g.world.mx.x, g.world.mx.y, g.world.mx.z,
                                 g.cellSize.x, g.cellSize.y, g.cellSize.z, g.cellSizeInv.x, g.cellSizeInv.y, g.cellSizeInv.z};
            std::memcpy(world, w, sizeof(w));
        }
        if (start != nullptr) std::memcpy(start, g.start.data(), g.start.size() * sizeof(int32_t));
        if (items != nullptr)  // input order indices, as the reference's grid holds its primitives
            for (size_t k = 0; k < g.items.size(); ++k) items[k] = order[static_cast<size_t>(g.items[k])];
    });
    return rc == 0 ? n : -1;
}

int64_t mrt_decode_texture(const char* path, int32_t* dims, uint8_t* texels) {
    int64_t n = -1;
    const int rc = guarded([&] {
        mrt::HTexture t;
        std::string err;
        if (!mrt::loadTextureFile(path != nullptr ? path : "", &t, &err)) throw std::runtime_error(err);
        n = static_cast<int64_t>(t.texels.size());
        if (dims != nullptr) {
            dims[0] = t.width;
            dims[1] = t.height;
            dims[2] = t.channels;
        }
        if (texels != nullptr) std::memcpy(texels, t.texels.data(), t.texels.size());
    });
    return rc == 0 ? n : -1;
}

int mrt_sample_tables(float* shader, float* sampler, float* trig) {
    return guarded([&] {
        std::vector<float> a, b, t;
        mrt::fillHaltonTable(&a, mrt::kSeedShaderTable);
        mrt::fillHaltonTable(&b, mrt::kSeedSamplerTable);
        mrt::fillHemisphereTrig(a, &t);
        if (shader != nullptr) std::memcpy(shader, a.data(), a.size() * sizeof(float));
        if (sampler != nullptr) std::memcpy(sampler, b.data(), b.size() * sizeof(float));
        if (trig != nullptr) std::memcpy(trig, t.data(), t.size() * sizeof(float));
    });
}

int mrt_get_tuning(const mrt_renderer* r, int32_t key, int32_t* value) {
    switch (key) {
        case 1: *value = r->ds.variant; return 0;
        case 2: *value = r->ds.cull; return 0;
        case 3: *value = r->overlap; return 0;
        case 7: *value = r->skipLast; return 0;
        case 5: *value = r->ds.anyOrder; return 0;
        case 6: *value = r->shadowGridPct; return 0;
        case 8: *value = r->ds.tailDonate; return 0;
        case 9: *value = r->refill; return 0;
        case 10: *value = r->ds.leanShade; return 0;
        case 11: *value = r->shadeGridPerCU; return 0;
        case 16: *value = r->ds.packet; return 0;
        case 17: *value = r->fuseL1Mode; return 0;
        case 27: *value = r->lastShadowRender; return 0;
        case 33: *value = r->genL1; return 0;
        case 34: *value = r->resolveAcc; return 0;
        case 35: *value = r->shadeWaitsShadow; return 0;
        case 28: *value = r->walkGridCap; return 0;
        default: break;
    }
    gLastError = "unknown tuning key";
    return -1;
}

int mrt_get_frame_stats(const mrt_renderer* r, mrt_frame_stats* s) {
    *s = r->last;
    return 0;
}

static void primaryHitsOne(mrt_renderer* r, int32_t* kind, int32_t* index, float* t);

int mrt_primary_hits(mrt_renderer* r, int32_t* kind, int32_t* index, float* t) {
    return guarded([&] {
        const size_t npx = static_cast<size_t>(r->cfg.width) * static_cast<size_t>(r->cfg.height);
        for (size_t i = 0; i < npx; ++i) {
            kind[i] = -1;
            index[i] = -1;
            t[i] = 0.0F;
        }
        for (int i = 0; i < groupSize(r); ++i) {  // a device group: every shard's pixels
            mrt_renderer* p = shardOf(r, i);
            MRT_HIP(hipSetDevice(p->device));
            primaryHitsOne(p, kind, index, t);
        }
        MRT_HIP(hipSetDevice(r->device));
    });
}

// the camera rays' first hits of this renderer's own pixels
static void primaryHitsOne(mrt_renderer* r, int32_t* kind, int32_t* index, float* t) {
    {
        using namespace mrt;
        hipStream_t st = r->stream;
        const auto& units = r->unitsByRank[static_cast<size_t>(r->rankIndex)];
        const auto& prefix = r->prefixByRank[static_cast<size_t>(r->rankIndex)];
        mrt_renderer::Pipe& pp = r->pipe;
        const int cap = pp.levels[1].cap;
        int32_t* dk = static_cast<int32_t*>(nullptr);
        int32_t* di = nullptr;
        float* dt = nullptr;
        MRT_HIP(hipMalloc(&dk, sizeof(int32_t) * static_cast<size_t>(cap)));
        MRT_HIP(hipMalloc(&di, sizeof(int32_t) * static_cast<size_t>(cap)));
        MRT_HIP(hipMalloc(&dt, sizeof(float) * static_cast<size_t>(cap)));
        std::vector<int32_t> hk(static_cast<size_t>(cap)), hi(static_cast<size_t>(cap));
        std::vector<float> ht(static_cast<size_t>(cap));
        try {
            for (int slot0 = 0; slot0 < r->nSlots; slot0 += cap) {
                const int n = std::min(cap, r->nSlots - slot0);
                MRT_HIP(hipMemsetAsync(pp.counters, 0, sizeof(int) * kNumCounters, st));
                r->countersClean = false;  // (left in use: the next pass resets them)
                RaygenArgs ra{};
                ra.cam = r->cam;
                ra.map = r->mapByRank[static_cast<size_t>(r->rankIndex)];
                ra.tables = r->ds.tables;
                ra.jitter = r->ds.jitterDraws;
                ra.width = r->cfg.width;
                ra.height = r->cfg.height;
                ra.slotBase = slot0;
                ra.nPaths = n;
                ra.spp = 1;
                ra.sppTotal = r->cfg.samplesPixel;
                setPixelSampler(r, &ra);
                ra.sampleBase = 0;
                launchRaygen(ra, pp.levels[1], pp.counters, st);
                launchTrace(r->ds, pp.levels[1], pp.counters, 1, pp.gstack, r->gdepth, pp.stats, false, r->traceThreads, st);
                launchDumpHits(pp.levels[1], n, dk, di, dt, st);
                MRT_HIP(hipMemcpyAsync(hk.data(), dk, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
                MRT_HIP(hipMemcpyAsync(hi.data(), di, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
                MRT_HIP(hipMemcpyAsync(ht.data(), dt, sizeof(float) * n, hipMemcpyDeviceToHost, st));
                MRT_HIP(hipStreamSynchronize(st));
                for (int q = 0; q < n; ++q) {
                    int x, y;
                    slotToXYHost(units, prefix, slot0 + q, &x, &y);
                    const size_t pix = static_cast<size_t>(y) * static_cast<size_t>(r->cfg.width) + static_cast<size_t>(x);
                    int32_t k = hk[static_cast<size_t>(q)], idx = hi[static_cast<size_t>(q)];
                    if (k == kTriangle) idx = r->triOrder[static_cast<size_t>(idx)];
                    if (k == kPlane) idx = r->planeOrder[static_cast<size_t>(idx)];
                    if (k == kSphere) idx = r->sphereOrder[static_cast<size_t>(idx)];
                    kind[pix] = k;
                    index[pix] = idx;
                    t[pix] = ht[static_cast<size_t>(q)];
                }
            }
        } catch (...) {
            (void)hipFree(dk);
            (void)hipFree(di);
            (void)hipFree(dt);
            throw;
        }
        (void)hipFree(dk);
        (void)hipFree(di);
        (void)hipFree(dt);
    }
}

}  // extern "C"

// ---- test and diagnostic entry points ---------------------------------------------------
namespace {
// scoped device buffer for the diagnostic entry points (not on the render path)
struct DevBuf {
    void* p = nullptr;
    explicit DevBuf(size_t bytes) { MRT_HIP(hipMalloc(&p, bytes == 0 ? 1 : bytes)); }
    ~DevBuf() { (void)hipFree(p); }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};
}  // namespace

extern "C" {

int mrt_kat_slab(const float* boxes, const float* orig, const float* dir, int32_t n, int32_t* out) {
    return guarded([&] {
        if (n <= 0) return;
        const size_t N = static_cast<size_t>(n);
        DevBuf b(N * 24), o(N * 12), d(N * 12), r(N * 12);
        MRT_HIP(hipMemcpy(b.p, boxes, N * 24, hipMemcpyHostToDevice));
        MRT_HIP(hipMemcpy(o.p, orig, N * 12, hipMemcpyHostToDevice));
        MRT_HIP(hipMemcpy(d.p, dir, N * 12, hipMemcpyHostToDevice));
        mrt::launchKatSlab(b.as<float>(), o.as<float>(), d.as<float>(), n, r.as<int32_t>(), nullptr);
        MRT_HIP(hipMemcpy(out, r.p, N * 12, hipMemcpyDeviceToHost));
    });
}

int mrt_kat_triangle(const float* tris, const float* orig, const float* dir, int32_t n, int32_t* hit, float* t) {
    return guarded([&] {
        if (n <= 0) return;
        const size_t N = static_cast<size_t>(n);
        DevBuf b(N * 36), o(N * 12), d(N * 12), h(N * 4), tt(N * 4);
        MRT_HIP(hipMemcpy(b.p, tris, N * 36, hipMemcpyHostToDevice));
        MRT_HIP(hipMemcpy(o.p, orig, N * 12, hipMemcpyHostToDevice));
        MRT_HIP(hipMemcpy(d.p, dir, N * 12, hipMemcpyHostToDevice));
        mrt::launchKatTriangle(b.as<float>(), o.as<float>(), d.as<float>(), n, h.as<int32_t>(), tt.as<float>(), nullptr);
        MRT_HIP(hipMemcpy(hit, h.p, N * 4, hipMemcpyDeviceToHost));
        MRT_HIP(hipMemcpy(t, tt.p, N * 4, hipMemcpyDeviceToHost));
    });
}

int mrt_trace_rays(mrt_renderer* r, const float* orig, const float* dir, const float* dist, const int32_t* src,
                   int32_t n, int32_t any, int32_t* kind, int32_t* index, float* t) {
    return guarded([&] {
        using namespace mrt;
        if (n <= 0) return;
        hipStream_t st = r->stream;
        mrt_renderer::Pipe& pp = r->pipe;
        Level& lv = pp.levels[1];
        const int cap = any ? lv.shadowCap : lv.cap;
        // input-order primitive -> BVH-order code (self-exclusion source), and back for the output
        auto inverse = [](const std::vector<int32_t>& order) {
            std::vector<int32_t> inv(order.size());
            for (size_t j = 0; j < order.size(); ++j) inv[static_cast<size_t>(order[j])] = static_cast<int32_t>(j);
            return inv;
        };
        const std::vector<int32_t> triInv = inverse(r->triOrder), planeInv = inverse(r->planeOrder),
                                   sphereInv = inverse(r->sphereOrder);
        std::vector<uint32_t> codes(static_cast<size_t>(n), kNoPrim);
        if (src != nullptr) {
            for (int32_t i = 0; i < n; ++i) {
                const int32_t k = src[2 * i], j = src[2 * i + 1];
                if (k == kTriangle) codes[i] = encodePrim(kTriangle, static_cast<uint32_t>(triInv.at(static_cast<size_t>(j))));
                if (k == kPlane) codes[i] = encodePrim(kPlane, static_cast<uint32_t>(planeInv.at(static_cast<size_t>(j))));
                if (k == kSphere) codes[i] = encodePrim(kSphere, static_cast<uint32_t>(sphereInv.at(static_cast<size_t>(j))));
                if (k == kLight) codes[i] = encodePrim(kLight, static_cast<uint32_t>(j));
            }
        }
        const size_t C = static_cast<size_t>(std::min(cap, n));
        DevBuf o(C * 12), d(C * 12), ds(C * 4), sc(C * 4);
        std::vector<float4> out(C);
        for (int32_t base = 0; base < n; base += static_cast<int32_t>(C)) {
            const int m = std::min(static_cast<int>(C), n - base);
            const size_t M = static_cast<size_t>(m);
            MRT_HIP(hipMemcpyAsync(o.p, orig + 3 * static_cast<size_t>(base), M * 12, hipMemcpyHostToDevice, st));
            MRT_HIP(hipMemcpyAsync(d.p, dir + 3 * static_cast<size_t>(base), M * 12, hipMemcpyHostToDevice, st));
            if (any) MRT_HIP(hipMemcpyAsync(ds.p, dist + base, M * 4, hipMemcpyHostToDevice, st));
            MRT_HIP(hipMemcpyAsync(sc.p, codes.data() + base, M * 4, hipMemcpyHostToDevice, st));
            MRT_HIP(hipMemsetAsync(pp.counters, 0, sizeof(int) * kNumCounters, st));
            r->countersClean = false;  // (left in use: the next pass resets them)
            launchLoadRays(lv, o.as<float>(), d.as<float>(), ds.as<float>(), sc.as<uint32_t>(), m, any != 0, pp.counters, st);
            if (any) {
                launchShadow(r->ds, lv, pp.counters, 1, pp.gstackShadow, r->gdepth, pp.stats, false, r->traceThreads, st);
                MRT_HIP(hipMemcpyAsync(out.data(), lv.sC, M * 16, hipMemcpyDeviceToHost, st));
            } else {
                launchTrace(r->ds, lv, pp.counters, 1, pp.gstack, r->gdepth, pp.stats, false, r->traceThreads, st);
                MRT_HIP(hipMemcpyAsync(out.data(), lv.hit, M * 16, hipMemcpyDeviceToHost, st));
            }
            MRT_HIP(hipStreamSynchronize(st));
            for (int q = 0; q < m; ++q) {
                const size_t i = static_cast<size_t>(base + q);
                const float4 h = out[static_cast<size_t>(q)];
                if (any) {
                    kind[i] = h.w != 0.0F ? 1 : 0;
                    index[i] = -1;
                    t[i] = 0.0F;
                    continue;
                }
                uint32_t code;
                std::memcpy(&code, &h.w, 4);
                int32_t k = static_cast<int32_t>(primKind(code)), idx = static_cast<int32_t>(primIndex(code));
                if (k == kTriangle) idx = r->triOrder[static_cast<size_t>(idx)];
                if (k == kPlane) idx = r->planeOrder[static_cast<size_t>(idx)];
                if (k == kSphere) idx = r->sphereOrder[static_cast<size_t>(idx)];
                if (k == kMiss) idx = -1;
                kind[i] = k;
                index[i] = idx;
                t[i] = h.x;
            }
        }
    });
}

}  // extern "C"

// ---- desktop C-ABI (C_wrapper.cpp:268-290) ---------------------------------------------------
namespace {
std::mutex gRendererMutex;
mrt_renderer* gRenderer = nullptr;

void workThread(::MobileRT::Config& config) {
    try {
        mrt_config c{};
        c.width = config.width;
        c.height = config.height;
        c.threads = config.threads;
        c.shader = config.shader;
        c.sceneIndex = config.sceneIndex;
        c.samplesPixel = config.samplesPixel;
        c.samplesLight = config.samplesLight;
        c.repeats = config.repeats;
        c.accelerator = config.accelerator;
        c.printStdOut = config.printStdOut ? 1 : 0;
        c.objFilePath = config.objFilePath.c_str();
        c.mtlFilePath = config.mtlFilePath.c_str();
        c.camFilePath = config.camFilePath.c_str();
        const char* md = std::getenv("MOBILERT_MAX_DEPTH");
        c.maxDepth = md != nullptr ? std::atoi(md) : 0;
        const char* dev = std::getenv("MOBILERT_DEVICE");
        c.device = dev != nullptr ? std::atoi(dev) : -1;
        c.rankCount = 1;
        // MOBILERT_DEVICES=0,1,...: the frame sharded over these GPUs (a device group)
        const std::vector<int32_t> devices = mrt::parseDeviceList(std::getenv("MOBILERT_DEVICES"));
        if (devices.size() > 1) {
            c.devices = devices.data();
            c.deviceCount = static_cast<int32_t>(devices.size());
            c.device = -1;
        }
        c.cull = 3;  // exact for every input
        c.progressive = 1;  // the UI polls config.bitmap while the frame renders
        const auto tc0 = std::chrono::steady_clock::now();
        mrt_renderer* r = createRenderer(&c);
        const auto tc1 = std::chrono::steady_clock::now();
        {
            std::lock_guard<std::mutex> lock(gRendererMutex);
            gRenderer = r;
        }
        int32_t repeats = config.repeats;
        const auto t0 = std::chrono::steady_clock::now();
        do {  // C_wrapper.cpp:227-233
            const size_t n = static_cast<size_t>(r->cfg.width) * static_cast<size_t>(r->cfg.height);
            MRT_HIP(hipMemcpyAsync(r->dBitmap, config.bitmap.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, r->stream));
            renderFrameDevice(r, r->dBitmap, nullptr, r->stream, config.bitmap.data());
            repeats--;
        } while (repeats > 0);
        const auto t1 = std::chrono::steady_clock::now();
        const double secs = std::chrono::duration<double>(t1 - t0).count();
        const uint64_t rays = r->totalRays.load();
        if (config.printStdOut) {
            std::printf("TRIANGLES = %lld\nLIGHTS = %lld\n", static_cast<long long>(r->nTri), static_cast<long long>(r->nLights));
            std::printf("Creating Time in secs = %f\n", std::chrono::duration<double>(tc1 - tc0).count());
            std::printf("Rendering Time in secs = %f\n", secs);
            std::printf("Casted rays = %llu\n", static_cast<unsigned long long>(rays));
            std::printf("width = %d\nheight = %d\n", config.width, config.height);
            std::printf("Total Millions rays per second = %f\n", (static_cast<double>(rays) / secs) / 1000000.0);
            std::fflush(stdout);
        }
        {
            std::lock_guard<std::mutex> lock(gRendererMutex);
            gRenderer = nullptr;
        }
        mrt_destroy(r);  // C_wrapper.cpp:265
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());  // C_wrapper.cpp:257-263
    }
}
}  // namespace

extern "C" void RayTrace(::MobileRT::Config& config, bool async) {
    if (async) {
        std::thread th(workThread, std::ref(config));
        th.detach();
    } else {
        workThread(config);
    }
}

extern "C" void stopRender() {
    std::lock_guard<std::mutex> lock(gRendererMutex);
    if (gRenderer != nullptr) stopAll(gRenderer);
}
