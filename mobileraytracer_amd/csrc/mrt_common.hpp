// mrt_common.hpp - numerics and record layouts shared by the host scene builder and
// the gfx950 kernels of the MobileRT render hot path.
//
// Every function here restates one piece of the reference's arithmetic with the SAME
// evaluation order, because the parity bar is bit-exact for primary-ray hit ids and for
// the Whitted Cornell image.  Compile every translation unit that
// includes this header with -ffp-contract=off and without -ffast-math.
//
// Reference citations are relative to /root/reference (TiagoMSSantos/MobileRayTracer).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#define MRT_HD __host__ __device__ __forceinline__

namespace mrt {

// ---- constants: app/MobileRT/Utils/Constants.hpp:22-79 --------------------------------
constexpr float kEpsilon = 1.0e-06F;       // Constants.hpp:22
constexpr float kEpsilonLarge = 1.0e-05F;  // Constants.hpp:28
constexpr float kRayLengthMax = 1.0e+30F;  // Constants.hpp:33
constexpr int kRayDepthMin = 1;            // Constants.hpp:39
constexpr int kRayDepthMaxDefault = 6;     // Constants.hpp:45 (a runtime parameter here)
constexpr int kNumberOfTiles = 256;        // Constants.hpp:50
constexpr uint32_t kArrayMask = 0xFFFFFu;  // Constants.hpp:70
constexpr uint32_t kArraySize = kArrayMask + 1u;
// glm::two_pi<float>(), glm::quarter_pi<float>(), glm::pi<float>() rounded to float.
constexpr float kTwoPi = 6.28318530717958647692528676655900576f;
constexpr float kQuarterPi = 0.785398163397448309615660845819875721f;
constexpr float kPi = 3.14159265358979323846264338327950288f;

// ---- vec3 with glm 1.0.1 scalar-path semantics ----------------
struct v3 {
    float x, y, z;
};

MRT_HD v3 mk(float x, float y, float z) { return v3{x, y, z}; }
MRT_HD v3 operator+(v3 a, v3 b) { return v3{a.x + b.x, a.y + b.y, a.z + b.z}; }
MRT_HD v3 operator-(v3 a, v3 b) { return v3{a.x - b.x, a.y - b.y, a.z - b.z}; }
MRT_HD v3 operator*(v3 a, v3 b) { return v3{a.x * b.x, a.y * b.y, a.z * b.z}; }
MRT_HD v3 operator*(v3 a, float s) { return v3{a.x * s, a.y * s, a.z * s}; }
MRT_HD v3 operator*(float s, v3 a) { return v3{s * a.x, s * a.y, s * a.z}; }
MRT_HD v3 operator/(v3 a, float s) { return v3{a.x / s, a.y / s, a.z / s}; }
MRT_HD v3 operator-(v3 a) { return v3{-a.x, -a.y, -a.z}; }
MRT_HD float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// glm::dot: tmp = a*b; return tmp.x + tmp.y + tmp.z  (left to right)
MRT_HD float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
// glm::cross
MRT_HD v3 cross(v3 x, v3 y) {
    return v3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
// glm::length = sqrt(dot(v, v)); glm::normalize = v * inversesqrt(dot(v, v)), inversesqrt(x) = 1/sqrt(x)
MRT_HD float length(v3 v) { return sqrtf(dot(v, v)); }
MRT_HD v3 normalize(v3 v) { return v * (1.0F / sqrtf(dot(v, v))); }
// glm::reflect(I, N) = I - N * dot(N, I) * 2
MRT_HD v3 reflect(v3 i, v3 n) { return i - (n * dot(n, i)) * 2.0F; }
// glm::refract(I, N, eta)
MRT_HD v3 refract(v3 i, v3 n, float eta) {
    const float d = dot(n, i);
    const float k = 1.0F - eta * eta * (1.0F - d * d);
    if (k >= 0.0F) {
        return (eta * i) - ((eta * d + sqrtf(k)) * n);
    }
    return v3{0.0F, 0.0F, 0.0F};
}
// libstdc++ std::min / std::max operand order (Appendix A.3): NaN semantics depend on it.
MRT_HD float stdmin(float a, float b) { return (b < a) ? b : a; }
MRT_HD float stdmax(float a, float b) { return (a < b) ? b : a; }
// glm::min / glm::max per component (same ternaries as libstdc++).
MRT_HD v3 vmin(v3 a, v3 b) { return v3{stdmin(a.x, b.x), stdmin(a.y, b.y), stdmin(a.z, b.z)}; }
MRT_HD v3 vmax(v3 a, v3 b) { return v3{stdmax(a.x, b.x), stdmax(a.y, b.y), stdmax(a.z, b.z)}; }
// Utils.hpp:278-281 hasPositiveValue = any(greaterThan(v, 0))
MRT_HD bool hasPositive(v3 v) { return v.x > 0.0F || v.y > 0.0F || v.z > 0.0F; }

// Perspective.cpp:40-46 fastArcTan
MRT_HD float fastArcTan(float value) {
    const float absValue = fabsf(value);
    const float a = kQuarterPi * value;
    const float b = value * (absValue - 1.0F);
    const float c = 0.2447F + (0.0663F * absValue);
    return a - b * c;
}

// Utils.cpp:66-90 incrementalAvg: float -> uint32 truncation, then pure uint32 arithmetic.
MRT_HD int32_t incrementalAvg(v3 sample, int32_t avg, int32_t numSample) {
    const uint32_t avgU = static_cast<uint32_t>(avg);
    const uint32_t n = static_cast<uint32_t>(numSample);
    const uint32_t lastR = avgU & 0xFFu;
    const uint32_t lastG = (avgU >> 8u) & 0xFFu;
    const uint32_t lastB = (avgU >> 16u) & 0xFFu;
    const uint32_t sR = static_cast<uint32_t>(sample.x * 255.0F);
    const uint32_t sG = static_cast<uint32_t>(sample.y * 255.0F);
    const uint32_t sB = static_cast<uint32_t>(sample.z * 255.0F);
    uint32_t cR = ((n - 1u) * lastR + sR) / n;
    uint32_t cG = ((n - 1u) * lastG + sG) / n;
    uint32_t cB = ((n - 1u) * lastB + sB) / n;
    cR = cR < 255u ? cR : 255u;
    cG = cG < 255u ? cG : 255u;
    cB = cB < 255u ? cB : 255u;
    return static_cast<int32_t>(0xFF000000u | cB << 16u | cG << 8u | cR);
}

// ---- deterministic sample streams -------
// The reference draws from shuffled 2^20-entry Halton tables through shared atomic cursors,
// which makes every run different.  Here every draw is a pure function of
// (pixel, global sample, vertex of the ray tree, purpose), so results are independent of
// thread scheduling, of chunking and of the GPU shard a pixel lands on.
MRT_HD uint32_t hash32(uint32_t x) {  // "lowbias32" integer mixer
    x ^= x >> 16u;
    x *= 0x7feb352du;
    x ^= x >> 15u;
    x *= 0x846ca68bu;
    x ^= x >> 16u;
    return x;
}
MRT_HD uint32_t pathKey(uint32_t pixelIndex, uint32_t globalSample) {
    return hash32(pixelIndex * 0x9E3779B9u ^ hash32(globalSample + 0x632BE5ABu));
}
// treeCode: 1 for the camera ray's vertex; child = code * 4 + slot (slot 1 diffuse,
// 2 specular, 3 transmission); 0 for the pixel sampler.  purpose: one of the kP* constants
// below.  The draws of one vertex are CONSECUTIVE table entries from a hashed start aligned to
// 8 entries, as the reference's sampler cursors hand out consecutive entries (Sampler.hpp:58-63,
// Shader.cpp:189-194); on the GPU every draw of a vertex (samplesLight 1) then comes from ONE
// 128-byte line of the interleaved table.
MRT_HD uint32_t sampleIndex(uint32_t key, uint32_t treeCode, uint32_t purpose) {
    return ((hash32(key ^ hash32(treeCode * 0x9E3779B9u + 0x7F4A7C15u)) & ~7u) + purpose) & kArrayMask;
}
// the 8-entry block every draw of a vertex comes from (sampleIndex without the purpose)
MRT_HD uint32_t sampleBlock(uint32_t key, uint32_t treeCode) {
    return (hash32(key ^ hash32(treeCode * 0x9E3779B9u + 0x7F4A7C15u)) & kArrayMask) >> 3;
}
// purposes
constexpr uint32_t kPJitterU = 0;   // pixel sampler, r1   (Renderer.cpp:137), tree code 0
constexpr uint32_t kPJitterV = 1;   // pixel sampler, r2   (Renderer.cpp:138), tree code 0
constexpr uint32_t kPRussian = 0;   // PathTracer RR       (PathTracer.cpp:89)
constexpr uint32_t kPHemi1 = 1;     // hemisphere r1       (Shader.cpp:190)
constexpr uint32_t kPHemi2 = 2;     // hemisphere r2       (Shader.cpp:191)
constexpr uint32_t kPLightBase = 3; // + 3*i + {0 pick, 1 r, 2 s} for light sample i
MRT_HD uint32_t purposeLightPick(int i) { return kPLightBase + 3u * static_cast<uint32_t>(i); }
MRT_HD uint32_t purposeLightR(int i) { return kPLightBase + 3u * static_cast<uint32_t>(i) + 1u; }
MRT_HD uint32_t purposeLightS(int i) { return kPLightBase + 3u * static_cast<uint32_t>(i) + 2u; }

// ---- hit / primitive encodings ---------------------------------------------------------
// kind order == the reference's category visiting order (Shader.cpp:104-111): planes,
// spheres, triangles, then lights.  Ties in t go to the earlier kind, then lower index.
enum PrimKind : uint32_t { kMiss = 0, kPlane = 1, kSphere = 2, kTriangle = 3, kLight = 4 };
MRT_HD uint32_t encodePrim(uint32_t kind, uint32_t index) { return (kind << 28u) | (index & 0x0FFFFFFFu); }
MRT_HD uint32_t primKind(uint32_t code) { return code >> 28u; }
MRT_HD uint32_t primIndex(uint32_t code) { return code & 0x0FFFFFFFu; }
constexpr uint32_t kNoPrim = 0u;

// BVH child reference: >= 0 inner node index; < 0 leaf: v = -ref-1, first = v >> 3, count = v & 7
MRT_HD int32_t leafRef(int32_t first, int32_t count) { return -((first << 3) | count) - 1; }
MRT_HD int32_t leafFirst(int32_t ref) { return (-ref - 1) >> 3; }
MRT_HD int32_t leafCount(int32_t ref) { return (-ref - 1) & 7; }

// Device BVH2 node: both children's boxes live in the parent (one 64-byte record per
// inner node), so one visit is 4 x 16-byte loads and tests the two boxes the reference
// tests at BVH.hpp:357-363.
struct alignas(16) GNode {
    float lminx, lminy, lminz, lmaxx;
    float lmaxy, lmaxz, rminx, rminy;
    float rminz, rmaxx, rmaxy, rmaxz;
    int32_t refL, refR;
    uint32_t coneL, coneR;  // cull words of the children (kConeNever: never culled)
};
static_assert(sizeof(GNode) == 64, "GNode must be 64 bytes");

// Walk-tree node ("quantized walk tree"): up to four children, each
// child's box as 16-bit coordinates on one scene-wide grid (real value origin + q * step per axis)
// rounded OUTWARD by one extra grid step (q[3c + a] = child c's min | max << 16 on axis a), and
// their references (kEmptyChild: no child): 64 bytes,
// four 16-byte loads per visit, about half the dependent visits of a BVH2.
constexpr int32_t kEmptyChild = 0x7FFFFFFE;
#ifndef MRT_WALK_WIDTH
#define MRT_WALK_WIDTH 4
#endif
constexpr int kWalkWidth = MRT_WALK_WIDTH;  // children per walk-tree node (4 or 8)
static_assert(kWalkWidth == 4 || kWalkWidth == 8, "walk width");
struct alignas(16) QNode4 {
    uint32_t q[3 * kWalkWidth];
    int32_t ref[kWalkWidth];
};
static_assert(sizeof(QNode4) == 16 * kWalkWidth, "QNode4: 16 bytes per child");
struct QGrid {
    float origin[3];
    float step[3];
};

// Cull word of a BVH2 child (GNode::coneL / coneR): what bounds the
// Moller-Trumbore t of every triangle below the child.  bits 0-17: the normal-line axis a
// (octahedral, 9 + 9 bits), bits 18-24: q = sin(psi) in 1/126 steps, rounded up, where every
// triangle normal n satisfies |n.a| >= cos(psi) (127: no such bound), bits 25-31: K in
// 2^(code/8) steps, rounded up, K >= |AB|_1 |AC|_1 / |AB x AC| of every triangle below (127: none).
constexpr uint32_t kConeNever = 0xFFFFFFFFu;
MRT_HD uint32_t coneQ(uint32_t w) { return (w >> 18) & 127u; }
MRT_HD uint32_t coneK(uint32_t w) { return w >> 25; }
MRT_HD v3 coneAxis(uint32_t w) {  // octahedral decode (not normalised: |a| in [1/sqrt(3), 1])
    float x = static_cast<float>(w & 511u) * (2.0F / 511.0F) - 1.0F;
    float y = static_cast<float>((w >> 9) & 511u) * (2.0F / 511.0F) - 1.0F;
    const float z = 1.0F - fabsf(x) - fabsf(y);
    if (z < 0.0F) {
        const float ox = x;
        x = (1.0F - fabsf(y)) * (ox >= 0.0F ? 1.0F : -1.0F);
        y = (1.0F - fabsf(ox)) * (y >= 0.0F ? 1.0F : -1.0F);
    }
    return v3{x, y, z};
}

// root box + root reference of one BVH (the reference tests the root box first,
// BVH.hpp:340-342)
struct GRoot {
    float bmin[3];
    float bmax[3];
    int32_t ref;     // inner index or leaf ref
    int32_t count;   // number of primitives (0 => empty BVH, BVH.hpp:328-330)
};

// x86 cvttss2si, the reference's float -> int32 conversion (static_cast<int32_t>): truncation,
// and INT32_MIN for NaN and out-of-range values (where the GPU's v_cvt_i32_f32 saturates)
MRT_HD int32_t x86Trunc(float f) {
    return (f >= -2147483648.0F && f < 2147483648.0F) ? static_cast<int32_t>(f) : static_cast<int32_t>(0x80000000u);
}

// RegularGrid<T> (RegularGrid.hpp) with gridSize 32 (Shader.cpp:57): one per primitive kind.
// Cell (x, y, z) is x + (y << 5) + (z << 10) (getCellIndex, gridShift 5); its primitives are
// items[start[c] .. start[c + 1]) (BVH-order indices, ascending input order; mrt_grid.cpp).
constexpr int kGridSize = 32;
constexpr int kGridShift = 5;  // bitCounter(gridSize - 1), RegularGrid.hpp:123,173-180
constexpr int kGridCells = kGridSize * kGridSize * kGridSize;
struct GGrid {
    float mn[3];   // worldBoundaries_ min (Scene::getBounds, Epsilon-widened)
    float cs[3];   // cellSize_
    float csi[3];  // cellSizeInverted_
    int32_t count; // primitives of this kind (0: the walk tests nothing)
    const int32_t* start;
    const int32_t* items;
};

// Camera parameters (Camera.cpp:14-19, Perspective.cpp:8-14)
struct GCamera {
    v3 position, direction, right, up;
    float hFov, vFov;  // perspective: radians; orthographic: half sizes (Orthographic.cpp:11-12)
    int32_t kind;      // 0 perspective, 1 orthographic
    int32_t pad;
};

}  // namespace mrt
