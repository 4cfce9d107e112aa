// mrt_grid.cpp - host build of the RegularGrid accelerator (Config::accelerator 2).
//
// RegularGrid<T> (app/MobileRT/Accelerators/RegularGrid.hpp) with gridSize 32 (Shader.cpp:56-61):
// the world box of the primitive kind (Scene::getBounds, Scene.hpp:51-62), the cell sizes and
// their inverses (RegularGrid.hpp:116-132), and every cell's primitive list, filled by the
// reference's own membership test (RegularGrid.hpp:215-289: the primitive's candidate cells from
// its box, then Triangle / Plane / Sphere::intersect(const AABB&)).  The arithmetic is restated in
// the reference's evaluation order (compiled with -ffp-contract=off), so cell lists are the
// reference's.  One deviation, shared with the oracle: the reference fills the grid from
// hardware_concurrency threads behind per-cell mutexes, so a cell's list order depends on lock
// order; here every list is in ascending input order (what one thread produces).
//
// The device walks the lists with the reference's 3D-DDA (mrt_device.hpp gridWalk).  Lists hold
// BVH-order primitive indices (the hit codes of every other accelerator); the CSR arrays are
// GGrid::start (kGridCells + 1) and GGrid::items.
#include "mrt_scene.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <thread>

namespace mrt {

namespace {

// Triangle::intersect(Intersection) (Triangle.cpp:63-95) for the box-diagonal ray of
// Triangle::intersect(const AABB&): no source primitive, length RayLengthMax
bool diagonalHits(const HTriangle& t, v3 o, v3 d) {
    const v3 p = cross(d, t.AC);
    const float det = dot(t.AB, p);
    if (std::fabs(det) < kEpsilon) return false;
    const float inv = 1.0F / det;
    const v3 s = o - t.A;
    const float u = inv * dot(s, p);
    if (u < 0.0F || u > 1.0F) return false;
    const v3 q = cross(s, t.AB);
    const float v = inv * dot(d, q);
    if (v < 0.0F || (u + v) > 1.0F) return false;
    const float dist = inv * dot(t.AC, q);
    return !(dist < kEpsilon || dist >= kRayLengthMax);
}

bool isNearFarInvalid(float nearT, float farT) { return (nearT > farT) || (farT < 0); }  // Triangle.cpp:132-134

// the lambdaIntersectRayAABB of Triangle.cpp:143-201: the half-line orig + t vec, t >= 0
bool edgeHitsBox(v3 orig, v3 vec, const HAABB& box) {
    float tNear = FLT_MIN;  // std::numeric_limits<float>::min()
    float tFar = FLT_MAX;
    for (int a = 0; a < 3; ++a) {
        const float o = comp(orig, a), d = comp(vec, a), mn = comp(box.mn, a), mx = comp(box.mx, a);
        if (std::fabs(d) < FLT_EPSILON) {
            if ((o < mn) || ((o + d) > mx)) return false;
        } else {
            float t1 = (mn - o) / d;
            float t2 = (mx - o) / d;
            if (t1 > t2) std::swap(t1, t2);
            tNear = stdmax(t1, tNear);  // std::max(t1[a], tNear)
            tFar = stdmin(t2, tFar);    // std::min(t2[a], tFar)
            if (isNearFarInvalid(tNear, tFar)) return false;
        }
    }
    return true;
}

}  // namespace

// Triangle::intersect(const AABB&) (Triangle.cpp:142-229)
bool boxIntersect(const HTriangle& t, const HAABB& box) {
    const v3 vec = box.mx - box.mn;
    const bool ab = edgeHitsBox(t.A, t.AB, box);
    const bool ac = edgeHitsBox(t.A, t.AC, box);
    const v3 b = t.A + t.AB;
    const v3 c = t.A + t.AC;
    const bool bc = edgeHitsBox(b, c - b, box);
    const bool ray = diagonalHits(t, box.mn, vec);
    const bool inside = std::fabs(dot(t.AB, cross(vec, t.AC))) < kEpsilon;  // lambdaIsOverTriangle
    return ab || ac || bc || ray || inside;
}

namespace {
// Plane::distance (Plane.cpp:117-138)
float planeDistance(const HPlane& p, v3 q) {
    const float d = p.normal.x * -p.point.x + p.normal.y * -p.point.y + p.normal.z * -p.point.z;
    const float num = p.normal.x * q.x + p.normal.y * q.y + p.normal.z * q.z + d;
    const float den = std::sqrt(p.normal.x * p.normal.x + p.normal.y * p.normal.y + p.normal.z * p.normal.z);
    return num / den;
}
}  // namespace

// Plane::intersect(const AABB&) (Plane.cpp:146-155)
bool boxIntersect(const HPlane& p, const HAABB& box) {
    const float dp = planeDistance(p, box.mx);
    const float dn = planeDistance(p, box.mn);
    return (dp <= 0 && dn >= 0) || (dp >= 0 && dn <= 0);
}

// Sphere::intersect(const AABB&) (Sphere.cpp:102-123)
bool boxIntersect(const HSphere& s, const HAABB& box) {
    float dmin = 0.0F;
    for (int a = 0; a < 3; ++a) {
        const float c = comp(s.center, a), lo = comp(box.mn, a), hi = comp(box.mx, a);
        if (c < lo) {
            dmin = dmin + (c - lo) * (c - lo);
        } else if (c > hi) {
            dmin = dmin + (c - hi) * (c - hi);
        }
    }
    return dmin <= s.sqRadius;
}

namespace {

// the candidate range of one axis (RegularGrid.hpp:239-244)
void candidateRange(float bmin, float bmax, float worldMin, float size, float reci, int* lo, int* hi) {
    int a = x86Trunc((bmin - worldMin) * reci);
    int b = x86Trunc((bmax - worldMin) * reci) + 1;
    a = std::max(0, a);
    b = std::min(b, kGridSize - 1);
    b = std::fabs(size) < FLT_EPSILON ? 0 : b;
    a = std::min(a, b);
    *lo = a;
    *hi = b;
}

}  // namespace

template <class T>
HGrid buildGrid(const std::vector<T>& prims, const std::vector<int32_t>& order) {
    HGrid g;
    const size_t n = prims.size();
    // input index -> BVH-order index: the reference's grid holds the primitives in input order
    std::vector<int32_t> bvhOf(n);
    for (size_t j = 0; j < n; ++j) bvhOf[static_cast<size_t>(order[j])] = static_cast<int32_t>(j);
    // Scene::getBounds (Scene.hpp:51-62, Scene.cpp:36-39)
    HAABB bounds{v3{kRayLengthMax, kRayLengthMax, kRayLengthMax}, v3{-kRayLengthMax, -kRayLengthMax, -kRayLengthMax}};
    for (size_t i = 0; i < n; ++i) {
        const HAABB b = aabbOf(prims[static_cast<size_t>(bvhOf[i])]);
        bounds = HAABB{vmin(b.mn, bounds.mn), vmax(b.mx, bounds.mx)};
    }
    const v3 eps{kEpsilon, kEpsilon, kEpsilon};
    g.world = HAABB{bounds.mn - eps, bounds.mx + eps};
    const v3 ext = g.world.mx - g.world.mn;
    const float gs = static_cast<float>(kGridSize);
    g.cellSizeInv = v3{gs / ext.x, gs / ext.y, gs / ext.z};  // RegularGrid.hpp:126-130
    g.cellSize = ext * (1.0F / gs);                           // RegularGrid.hpp:132
    g.count = static_cast<int32_t>(n);
    g.start.assign(static_cast<size_t>(kGridCells) + 1, 0);
    if (n == 0) return g;

    // addPrimitivesThreadWork (RegularGrid.hpp:216-289)
    const v3 wmin = g.world.mn, size = g.world.mx - g.world.mn;
    const float dx = size.x / static_cast<float>(kGridSize);
    const float dy = size.y / static_cast<float>(kGridSize);
    const float dz = size.z / static_cast<float>(kGridSize);
    const float dxR = dx > 0 ? 1.0F / dx : 1.0F;
    const float dyR = dy > 0 ? 1.0F / dy : 1.0F;
    const float dzR = dz > 0 ? 1.0F / dz : 1.0F;
    const unsigned hw = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
    const size_t workers = std::min<size_t>(hw, (n + 4095) / 4096);
    // contiguous input ranges per worker; (cell, BVH index) pairs in input order
    std::vector<std::vector<std::pair<int32_t, int32_t>>> parts(workers);
    auto work = [&](size_t w) {
        const size_t i0 = n * w / workers, i1 = n * (w + 1) / workers;
        std::vector<std::pair<int32_t, int32_t>>& out = parts[w];
        for (size_t i = i0; i < i1; ++i) {
            const T& p = prims[static_cast<size_t>(bvhOf[i])];
            const HAABB b = aabbOf(p);
            int x1, x2, y1, y2, z1, z2;
            candidateRange(b.mn.x, b.mx.x, wmin.x, size.x, dxR, &x1, &x2);
            candidateRange(b.mn.y, b.mx.y, wmin.y, size.y, dyR, &y1, &y2);
            candidateRange(b.mn.z, b.mx.z, wmin.z, size.z, dzR, &z1, &z2);
            for (int x = x1; x <= x2; ++x) {
                for (int y = y1; y <= y2; ++y) {
                    for (int z = z1; z <= z2; ++z) {
                        const int32_t idx = x + y * kGridSize + z * kGridSize * kGridSize;
                        const v3 pos{wmin.x + static_cast<float>(x) * dx, wmin.y + static_cast<float>(y) * dy,
                                     wmin.z + static_cast<float>(z) * dz};
                        const HAABB cell{pos, pos + v3{dx, dy, dz}};
                        if (boxIntersect(p, cell)) out.emplace_back(idx, bvhOf[i]);
                    }
                }
            }
        }
    };
    std::vector<std::thread> pool;
    for (size_t w = 1; w < workers; ++w) pool.emplace_back(work, w);
    work(0);
    for (std::thread& t : pool) t.join();
    // CSR by cell, stable in input order (parts are consecutive input ranges)
    for (const auto& part : parts)
        for (const auto& e : part) ++g.start[static_cast<size_t>(e.first) + 1];
    for (size_t c = 0; c < static_cast<size_t>(kGridCells); ++c) g.start[c + 1] += g.start[c];
    g.items.assign(static_cast<size_t>(g.start[kGridCells]), 0);
    std::vector<int32_t> fill(g.start.begin(), g.start.end() - 1);
    for (const auto& part : parts)
        for (const auto& e : part) g.items[static_cast<size_t>(fill[static_cast<size_t>(e.first)]++)] = e.second;
    return g;
}

template HGrid buildGrid<HTriangle>(const std::vector<HTriangle>&, const std::vector<int32_t>&);
template HGrid buildGrid<HPlane>(const std::vector<HPlane>&, const std::vector<int32_t>&);
template HGrid buildGrid<HSphere>(const std::vector<HSphere>&, const std::vector<int32_t>&);

}  // namespace mrt
