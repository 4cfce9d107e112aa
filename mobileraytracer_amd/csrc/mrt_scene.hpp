// mrt_scene.hpp - host-side scene assembly for the MI355X render path.
//
// This is the "Shader constructor" half of the reference (Shader.cpp:33-77): it gathers
// planes / spheres / triangles / lights / materials, builds one BVH per primitive kind
// with the reference's build algorithm (BVH.hpp:126-283), generates the two sample tables
// (Utils.hpp:209-218 with fixed seeds) and flattens everything into the 16-byte aligned
// records the gfx950 kernels read.  None of this runs inside the timed render window.
#pragma once

#include "mrt_common.hpp"

#include <functional>
#include <istream>
#include <string>
#include <array>
#include <vector>

namespace mrt {

struct v2 {
    float x, y;
};

// Material.hpp:18-43
struct HMaterial {
    v3 Le{0, 0, 0}, Kd{0, 0, 0}, Ks{0, 0, 0}, Kt{0, 0, 0};
    float ior{1.0F};
    std::string texture;  // map_Kd file name ("" = none)
    int32_t texId{-1};    // index into HScene::textures (-1: none)
};

// Texture (Texture.hpp): 8-bit channels as stb_image returns them (Texture.cpp:83-114)
struct HTexture {
    int32_t width{0}, height{0}, channels{0};
    std::vector<uint8_t> texels;
};
// mrt_texture.cpp: PNG bytes -> texture (stb_image's conventions); false + err when unsupported
bool decodePng(const std::vector<uint8_t>& file, HTexture* out, std::string* err);
bool loadTextureFile(const std::string& path, HTexture* out, std::string* err);
bool materialEqual(const HMaterial& a, const HMaterial& b);  // Material.cpp:106-115

// Triangle.hpp:18-27 (field order kept: AC, AB, A, normals, texcoords, material)
struct HTriangle {
    v3 AC, AB, A;
    v3 nA, nB, nC;
    v2 tA{-1, -1}, tB{-1, -1}, tC{-1, -1};
    int32_t mat{-1};
};
// Triangle::Builder (Triangle.cpp:328-339) + Triangle ctor normalisation (Triangle.cpp:14-26)
HTriangle makeTriangle(v3 a, v3 b, v3 c);
HTriangle makeTriangle(v3 a, v3 b, v3 c, v3 na, v3 nb, v3 nc, v2 ta, v2 tb, v2 tc, int32_t mat);

struct HPlane {  // Plane.cpp:14-19
    v3 normal, point;
    int32_t mat;
};
HPlane makePlane(v3 point, v3 normal, int32_t mat);

struct HSphere {  // Sphere.cpp:14-19
    v3 center;
    float sqRadius;
    int32_t mat;
};
HSphere makeSphere(v3 center, float radius, int32_t mat);

enum LightKind : int32_t { kPointLight = 0, kAreaLight = 1 };
struct HLight {  // PointLight.cpp / AreaLight.cpp
    int32_t kind;
    HMaterial radiance;
    v3 position;  // point light
    HTriangle tri; // area light
};

struct HAABB {
    v3 mn, mx;
};

struct HScene {
    std::vector<HPlane> planes;
    std::vector<HSphere> spheres;
    std::vector<HTriangle> triangles;
    std::vector<HLight> lights;
    std::vector<HMaterial> materials;
    std::vector<HTexture> textures;  // map_Kd images, cached by file name (OBJLoader.cpp:224-242)
};

// Reference BVH node (BVH.hpp:56-60): box, indexOffset (leaf: first prim; inner: left),
// numPrimitives (> 0 => leaf)
struct HBVHNode {
    HAABB box;
    int32_t indexOffset;
    int32_t numPrimitives;
};

// ---- scenes / loaders ------------------------------------------------------------------
HScene cornellBoxScene();                                     // Scenes.cpp:63-137 (scene 0)
HScene builtinScene(int index);                               // C_wrapper.cpp:76-99: scenes 0-3
GCamera builtinCamera(int index, float ratio);                // their cameras (Scenes.cpp)
v3 builtinMaxPoint(int index);                                // DepthMap maxDist (C_wrapper.cpp:79-131)
GCamera makeOrthographic(v3 position, v3 lookAt, v3 up, float sizeH, float sizeV);
GCamera cornellBoxCamera(float ratio);                        // Scenes.cpp:139-150
GCamera makePerspective(v3 position, v3 lookAt, v3 up, float hFovDeg, float vFovDeg);
// CameraFactory.cpp + PerspectiveLoader.cpp:18-64 (position.x negated, hFov = fov.u * ratio)
bool loadCameraFile(const std::string& path, float ratio, GCamera* out, std::string* err);
// the same from a stream (the Android front end hands the .cam text over, JNI_layer.cpp:994-1063)
bool loadCameraStream(std::istream& in, float ratio, GCamera* out, std::string* err, const std::string& name = "");
// OBJLoader.cpp:18-497 (+ tinyobjloader v1.0.7 parsing / fan triangulation); fills in file order
bool loadObjScene(const std::string& objPath, const std::string& mtlPath, HScene* scene, std::string* err);
// the same from streams; map_Kd textures come from textureSource(name) (false: not available)
using TextureSource = std::function<bool(const std::string&, HTexture*)>;
bool loadObjStreams(std::istream& obj, std::istream* mtl, const TextureSource& textureSource, HScene* scene,
                    std::string* err);

// ---- acceleration structure ------------------------------------------------------------
// libstdc++ std::partition (bidirectional overload), restated so the build is pinned.
template <class It, class Pred>
It pinnedPartition(It first, It last, Pred pred) {
    while (true) {
        while (true) {
            if (first == last) return first;
            if (pred(*first)) ++first; else break;
        }
        --last;
        while (true) {
            if (first == last) return first;
            if (!pred(*last)) --last; else break;
        }
        auto tmp = *first;
        *first = *last;
        *last = tmp;
        ++first;
    }
}

HAABB aabbOf(const HTriangle& t);  // Triangle.cpp:116-123
HAABB aabbOf(const HPlane& p);     // Plane.cpp:79-109
HAABB aabbOf(const HSphere& s);    // Sphere.cpp:88-94
bool aabbIntersect(const HAABB& b, v3 origin, v3 dir);  // AABB.cpp:34-54 (host KAT helper)

// Builds the reference BVH over `prims` (permuted in place to leaf order).  Returns nodes
// in the reference numbering.  `order` receives the original index of every permuted prim.
template <class T>
std::vector<HBVHNode> buildBVH(std::vector<T>* prims, std::vector<int32_t>* order);

// Converts reference nodes to the device child-box layout: the first topCount inner nodes
// breadth-first (the trace kernel stages them in LDS), the rest depth-first pre-order.
// cones: the cull word of every reference node (triangleConeWords), or null (never culled).
void toDeviceBVH(const std::vector<HBVHNode>& nodes, size_t numPrims, std::vector<GNode>* out, GRoot* root,
                 int topCount = 0, int* topPlaced = nullptr, const std::vector<uint32_t>* cones = nullptr);
// The walk tree collapsed to 4-wide nodes (each node's children: its BVH2 children, the inner one
// of largest area replaced by its own children while fewer than four), quantized like
// Quantizer (mrt_scene.cpp) and numbered as toDeviceBVH numbers (the first topCount breadth-first).  Fills
// root (box of nodes[0], reference into out); false when a box or the grid is not finite.
// nodeCost: the collapse's cost of each BVH2 node as a wide node (null: its surface area).
bool toQuantizedBVH4(const std::vector<HBVHNode>& nodes, size_t numPrims, GRoot* root, int topCount, int* topPlaced,
                     QGrid* grid, std::vector<QNode4>* out, std::vector<int32_t>* bvh2Of = nullptr,
                     const std::vector<double>* nodeCost = nullptr);
// The frame's own ray distribution as collapse costs (MOBILERT_COLLAPSE=rays, an A/B setting): a
// sample of the frame's walked rays - camera rays over a pixel grid, then per hit a shadow ray to a
// random point of a random light and the PathTracer's children (cosine bounce, mirror reflection)
// up to maxDepth, traced on the host - and cost[i] = the weighted number of sample rays whose
// half-line passes node i's box (the exact walk visits every wide node it passes), plus 1 % of the
// node's share of the root's area as a floor.  Any cost gives an exact walk: only the collapse changes.
std::vector<double> frameRayNodeCosts(const std::vector<HBVHNode>& nodes, const HScene& sc, const GCamera& cam,
                                      int width, int height, int maxDepth);
// frameRayNodeCosts' sample: the rays (origin, direction, weight) traced on the host over `nodes`
struct SampleRay {
    v3 o, d;
    float w;
};
std::vector<SampleRay> sampleFrameRays(const std::vector<HBVHNode>& nodes, const HScene& sc, const GCamera& cam,
                                       int maxDepth);
// frameRayNodeCosts over a given sample
std::vector<double> sampleRayNodeCosts(const std::vector<HBVHNode>& nodes, const std::vector<SampleRay>& rays);
// The walk tree's BVH2 rotated where that lowers its 4-wide collapse's cost under the sample
// (sampleRayNodeCosts' node cost), up to `sweeps` sweeps; same leaves, exact-union inner boxes, no
// subtree taller than in `in`.
std::vector<HBVHNode> rotateForRays(const std::vector<HBVHNode>& in, const std::vector<SampleRay>& rays, int sweeps);
// A tree over the same leaves (primitive ranges and boxes) as the reference tree `ref`, grouped
// by a full-sweep SAH; its inner boxes are exact unions of the leaf boxes (reference numbering:
// node 0 the root, an inner node's children at indexOffset and indexOffset + 1).
std::vector<HBVHNode> rebuildOverLeaves(const std::vector<HBVHNode>& ref, int weight = 0);
// The same tree with its summed inner-node area lowered by insertion-based optimisation (at most
// `rounds` rounds; leaves and exact-union boxes kept, reference numbering; bounded: no insertion
// makes the tree higher than it was)
std::vector<HBVHNode> optimizeOverLeaves(const std::vector<HBVHNode>& tree, int rounds, bool bounded = true);
// The walk tree over the reference tree's leaves: rebuildOverLeaves (weight 2), then
// optimizeOverLeaves (MOBILERT_TREE_OPT rounds, default kTreeOptRounds) where it lowers the wide
// tree's summed area without adding wide levels, then rotations that lower the wide area directly
// (MOBILERT_TREE_ROT sweeps, default kTreeRotSweeps); the reference tree itself with
// MOBILERT_WALK_TREE=0.  Built once per reference tree and settings in a process (the last
// kTreeCacheScenes kept).
constexpr int kTreeOptRounds = 100;
constexpr int kTreeRotSweeps = 1;
constexpr size_t kTreeCacheScenes = 4;
std::vector<HBVHNode> walkTreeOver(const std::vector<HBVHNode>& ref);
// The cull word (mrt_common.hpp) of every node of a triangle BVH built by buildBVH over tris
// (already in BVH order): the normal-line cone and the conditioning bound K of its triangles.
std::vector<uint32_t> triangleConeWords(const std::vector<HBVHNode>& nodes, const std::vector<HTriangle>& tris);
// The certified-cull record of a set of triangles [lo, hi) inside box (the exact mode's leaf cull,
// mrt_trace_ww.hpp leafKey): out = {a'.x, a'.y, a'.z, q, Kc, D} with a' = a cos(psi) for a normal-line
// cone (axis a, half-angle psi) holding every triangle's normal, q >= sin(psi), Kc >= 2^-18 * 1.001 *
// max(1, |AB|_1 |AC|_1 / |AB x AC|), D >= 2.0002 * half diagonal + 2^-20 (|centre|_1 + half diagonal).
// No bound (degenerate triangle, cone wider than 90 degrees): {0, 0, 0, 1, 0, 0}, which never culls.
void leafCullRecord(const std::vector<HTriangle>& tris, size_t lo, size_t hi, const HAABB& box, float out[6]);
// The same over several triangle ranges, with D covering a box of half diagonal hd around centre ctr.
void cullRecord(const std::vector<HTriangle>& tris, const std::vector<std::array<int32_t, 2>>& ranges,
                const double ctr[3], double hd, float out[6]);

// RegularGrid<T> build (mrt_grid.cpp): prims in BVH order, order[j] = input index of prims[j]
struct HGrid {
    HAABB world;
    v3 cellSize, cellSizeInv;
    int32_t count = 0;
    std::vector<int32_t> start, items;  // CSR over kGridCells cells
};
// the primitives' box tests that decide cell membership (Triangle.cpp:142-229, Plane.cpp:146-155,
// Sphere.cpp:102-123)
bool boxIntersect(const HTriangle& t, const HAABB& box);
bool boxIntersect(const HPlane& p, const HAABB& box);
bool boxIntersect(const HSphere& s, const HAABB& box);
template <class T>
HGrid buildGrid(const std::vector<T>& prims, const std::vector<int32_t>& order);

// Utils.cpp:43-53 haltonSequence
float haltonSequence(uint32_t index, uint32_t base);
// Utils.hpp:209-218 with std::mt19937(seed) instead of random_device
void fillHaltonTable(std::vector<float>* table, uint32_t seed);
// Shader::getCosineSampleHemisphere (Shader.cpp:188-216) takes cos and sin of phi = 2 pi r1 with
// r1 a shader-table entry, through the platform's libm (cosf / sinf).  They depend on the entry
// alone, so the host evaluates them once per entry: out[2 i] = cos, out[2 i + 1] = sin.
void fillHemisphereTrig(const std::vector<float>& shaderTable, std::vector<float>* out);
constexpr uint32_t kSeedShaderTable = 0x4D525400u;   // Shader.cpp:23,37
constexpr uint32_t kSeedSamplerTable = 0x4D525401u;  // StaticHaltonSeq.cpp:7-22

// MOBILERT_DEVICES ("0,1,2,3") -> the device group's ordinals (mrt_config.devices); null -> {}
std::vector<int32_t> parseDeviceList(const char* s);

}  // namespace mrt
