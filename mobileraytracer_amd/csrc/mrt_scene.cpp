// mrt_scene.cpp - host-side scene assembly (see mrt_scene.hpp).
#include "mrt_scene.hpp"

#include <algorithm>
#include <limits>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <fstream>
#include <memory>
#include <mutex>
#include <queue>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>

namespace mrt {

// ---- materials ----------------------------------------------------------------------------
namespace {
bool feq(float a, float b) { return std::fabs(a - b) < kEpsilon; }  // Utils.cpp:133-137
bool veq(v3 a, v3 b) { return feq(a.x, b.x) && feq(a.y, b.y) && feq(a.z, b.z); }
}  // namespace

bool materialEqual(const HMaterial& a, const HMaterial& b) {
    return veq(a.Kd, b.Kd) && veq(a.Ks, b.Ks) && veq(a.Kt, b.Kt) && veq(a.Le, b.Le) && feq(a.ior, b.ior) &&
           a.texture == b.texture;
}

static HMaterial material(v3 kd, v3 ks = v3{0, 0, 0}, v3 kt = v3{0, 0, 0}, float ior = 1.0F, v3 le = v3{0, 0, 0}) {
    HMaterial m;
    m.Kd = kd;
    m.Ks = ks;
    m.Kt = kt;
    m.ior = ior;
    m.Le = le;
    return m;
}

// ---- primitives -----------------------------------------------------------------------
HTriangle makeTriangle(v3 a, v3 b, v3 c) {
    const v3 ac = c - a;
    const v3 ab = b - a;
    const v3 n = normalize(cross(ac, ab));  // Triangle.cpp:336-338
    return makeTriangle(a, b, c, n, n, n, v2{-1, -1}, v2{-1, -1}, v2{-1, -1}, -1);
}

HTriangle makeTriangle(v3 a, v3 b, v3 c, v3 na, v3 nb, v3 nc, v2 ta, v2 tb, v2 tc, int32_t mat) {
    HTriangle t;
    t.AC = c - a;
    t.AB = b - a;
    t.A = a;
    t.nA = normalize(na);  // Triangle.cpp:18-20: the ctor normalises again
    t.nB = normalize(nb);
    t.nC = normalize(nc);
    t.tA = ta;
    t.tB = tb;
    t.tC = tc;
    t.mat = mat;
    return t;
}

HPlane makePlane(v3 point, v3 normal, int32_t mat) { return HPlane{normalize(normal), point, mat}; }

HSphere makeSphere(v3 center, float radius, int32_t mat) { return HSphere{center, radius * radius, mat}; }

HAABB aabbOf(const HTriangle& t) {
    const v3 b = t.A + t.AB;
    const v3 c = t.A + t.AC;
    return HAABB{vmin(t.A, vmin(b, c)), vmax(t.A, vmax(b, c))};
}

HAABB aabbOf(const HPlane& p) {
    v3 right{0, 0, 0};  // Plane.cpp:79-96 getRightVector
    const v3 n = p.normal;
    if (n.x >= 1) {
        right = v3{0, 1, 1};
    } else if (n.y >= 1) {
        right = v3{1, 0, 1};
    } else if (n.z >= 1) {
        right = v3{1, 1, 0};
    } else if (n.x <= -1) {
        right = v3{0, 1, 1};
    } else if (n.y <= -1) {
        right = v3{1, 0, 1};
    } else if (n.z <= -1) {
        right = v3{1, 1, 0};
    }
    right = normalize(right);
    return HAABB{p.point + right * -100.0F, p.point + right * 100.0F};
}

HAABB aabbOf(const HSphere& s) {
    const float r = std::sqrt(s.sqRadius);
    return HAABB{v3{s.center.x - r, s.center.y - r, s.center.z - r}, v3{s.center.x + r, s.center.y + r, s.center.z + r}};
}

bool aabbIntersect(const HAABB& b, v3 o, v3 d) {
    const float invX = 1.0F / d.x;
    const float t1x = (b.mn.x - o.x) * invX;
    const float t2x = (b.mx.x - o.x) * invX;
    float tMin = stdmin(t1x, t2x);
    float tMax = stdmax(t1x, t2x);
    for (int axis = 1; axis < 3; ++axis) {
        const float inv = 1.0F / comp(d, axis);
        const float org = comp(o, axis);
        const float t1 = (comp(b.mn, axis) - org) * inv;
        const float t2 = (comp(b.mx, axis) - org) * inv;
        tMin = stdmax(tMin, stdmin(t1, t2));
        tMax = stdmin(tMax, stdmax(t1, t2));
    }
    return tMax >= stdmax(tMin, 0.0F);
}

// ---- built-in Cornell box (Scenes.cpp:19-150) -----------------------------------------
namespace {
// Scenes.cpp:19-58 materials
const HMaterial kLightMat = material(v3{0, 0, 0}, v3{0, 0, 0}, v3{0, 0, 0}, 1.0F, v3{0.9F, 0.9F, 0.9F});
const HMaterial kMirrorMat = material(v3{0, 0, 0}, v3{0.9F, 0.9F, 0.9F}, v3{0, 0, 0}, 1.0F);
const HMaterial kTransmissionMat = material(v3{0, 0, 0}, v3{0, 0, 0}, v3{0.9F, 0.9F, 0.9F}, 1.9F);
const HMaterial kLightGrayMat = material(v3{0.7F, 0.7F, 0.7F});
const HMaterial kRedMat = material(v3{0.9F, 0.0F, 0.0F});
const HMaterial kYellowMat = material(v3{0.9F, 0.9F, 0.0F});
const HMaterial kGreenMat = material(v3{0.0F, 0.9F, 0.0F});
const HMaterial kBlueMat = material(v3{0.0F, 0.0F, 0.9F});
const HMaterial kSandMat = material(v3{0.914F, 0.723F, 0.531F});
const HMaterial kLightBlueMat = material(v3{0.0F, 0.9F, 0.9F});

void addTriangle(HScene* s, v3 a, v3 b, v3 c, const HMaterial& m) {
    HTriangle tri = makeTriangle(a, b, c);
    tri.mat = static_cast<int32_t>(s->materials.size());
    s->triangles.push_back(tri);
    s->materials.push_back(m);
}

void addSphere(HScene* s, v3 c, float r, const HMaterial& m) {
    s->spheres.push_back(makeSphere(c, r, static_cast<int32_t>(s->materials.size())));
    s->materials.push_back(m);
}

void addPlane(HScene* s, v3 p, v3 n, const HMaterial& m) {
    s->planes.push_back(makePlane(p, n, static_cast<int32_t>(s->materials.size())));
    s->materials.push_back(m);
}

void cornellBoxWalls(HScene* s) {  // Scenes.cpp:63-107
    const v3 back{0, 0, 1}, front{0, 0, -1}, bottom{0, -1, 0}, top{0, 1, 0};
    addPlane(s, back, front, kLightGrayMat);
    addPlane(s, v3{0.0F, 0.0F, -3.5F}, v3{0.0F, 0.0F, 1.0F}, kLightBlueMat);
    addPlane(s, bottom, top, kLightGrayMat);
    addPlane(s, top, bottom, kLightGrayMat);
    addPlane(s, v3{-1.0F, 0.0F, 0.0F}, v3{1.0F, 0.0F, 0.0F}, kRedMat);
    addPlane(s, v3{1.0F, 0.0F, 0.0F}, v3{-1.0F, 0.0F, 0.0F}, kBlueMat);
}

HLight pointLight(v3 p) {
    HLight l;
    l.kind = kPointLight;
    l.radiance = kLightMat;
    l.position = p;
    return l;
}
}  // namespace

HScene cornellBoxScene() {  // Scenes.cpp:109-137
    HScene s;
    s.lights.push_back(pointLight(v3{0.0F, 0.99F, 0.0F}));
    addTriangle(&s, v3{0.5F, -0.5F, 0.99F}, v3{0.5F, 0.5F, 1.001F}, v3{-0.5F, -0.5F, 0.99F}, kYellowMat);
    addSphere(&s, v3{0.45F, -0.65F, 0.4F}, 0.35F, kMirrorMat);
    addSphere(&s, v3{-0.45F, -0.1F, 0.0F}, 0.35F, kGreenMat);
    cornellBoxWalls(&s);
    return s;
}

HScene builtinScene(int index) {
    HScene s;
    switch (index) {
        case 0:
            return cornellBoxScene();
        case 1:  // spheres_Scene (Scenes.cpp:227-249): no lights
            addSphere(&s, v3{4.0F, 4.0F, 4.0F}, 4.0F, kRedMat);
            addTriangle(&s, v3{0.0F, 10.0F, 10.0F}, v3{0.0F, 0.0F, 10.0F}, v3{10.0F, 0.0F, 10.0F}, kSandMat);
            return s;
        case 2: {  // cornellBox2_Scene (Scenes.cpp:152-224): two area lights, transmission
            const v3 quad[2][3] = {{v3{-0.25F, 0.99F, -0.25F}, v3{0.25F, 0.99F, -0.25F}, v3{0.25F, 0.99F, 0.25F}},
                                   {v3{0.25F, 0.99F, 0.25F}, v3{-0.25F, 0.99F, 0.25F}, v3{-0.25F, 0.99F, -0.25F}}};
            for (const auto& q : quad) {
                HLight l;
                l.kind = kAreaLight;
                l.radiance = kLightMat;
                l.position = v3{0, 0, 0};
                l.tri = makeTriangle(q[0], q[1], q[2]);
                l.tri.mat = -1;
                s.lights.push_back(l);
            }
            addTriangle(&s, v3{0.5F, -0.5F, 0.99F}, v3{0.5F, 0.5F, 1.001F}, v3{-0.5F, -0.5F, 0.99F}, kYellowMat);
            addTriangle(&s, v3{-0.5F, 0.5F, 0.99F}, v3{-0.5F, -0.5F, 0.99F}, v3{0.5F, 0.5F, 0.99F}, kGreenMat);
            addSphere(&s, v3{0.45F, -0.65F, 0.4F}, 0.35F, kMirrorMat);
            addSphere(&s, v3{-0.4F, -0.3F, 0.0F}, 0.35F, kTransmissionMat);
            cornellBoxWalls(&s);
            return s;
        }
        default:  // 3: spheres2_Scene (Scenes.cpp:264-289)
            s.lights.push_back(pointLight(v3{0.0F, 15.0F, 4.0F}));
            addSphere(&s, v3{-1.0F, 1.0F, 6.0F}, 1.0F, kRedMat);
            addSphere(&s, v3{-0.5F, 2.0F, 5.0F}, 0.3F, kBlueMat);
            addSphere(&s, v3{0.0F, 2.0F, 7.0F}, 1.0F, kMirrorMat);
            addSphere(&s, v3{0.5F, 0.5F, 5.0F}, 0.2F, kYellowMat);
            addSphere(&s, v3{1.0F, 0.5F, 4.5F}, 0.5F, kGreenMat);
            addPlane(&s, v3{0.0F, 0.0F, 0.0F}, v3{0.0F, 1.0F, 0.0F}, kSandMat);
            return s;
    }
}

GCamera builtinCamera(int index, float ratio) {
    switch (index) {
        case 1:  // spheres_Cam (Scenes.cpp:251-262)
            return makeOrthographic(v3{0.0F, 1.0F, -10.0F}, v3{0.0F, 1.0F, 7.0F}, v3{0.0F, 1.0F, 0.0F}, 10.0F * ratio,
                                    10.0F);
        case 3:  // spheres2_Cam (Scenes.cpp:291-302)
            return makePerspective(v3{0.0F, 0.5F, 1.0F}, v3{0.0F, 0.0F, 7.0F}, v3{0.0F, 1.0F, 0.0F}, 60.0F * ratio, 60.0F);
        default:  // 0, 2: cornellBox_Cam
            return cornellBoxCamera(ratio);
    }
}

v3 builtinMaxPoint(int index) {  // C_wrapper.cpp:79-131 maxDist (DepthMap)
    return (index == 1 || index == 3) ? v3{8.0F, 8.0F, 8.0F} : v3{1.0F, 1.0F, 1.0F};
}

GCamera makeOrthographic(v3 position, v3 lookAt, v3 up, float sizeH, float sizeV) {  // Orthographic.cpp:7-13
    GCamera c{};
    c.position = position;
    c.direction = normalize(lookAt - position);  // Camera.cpp:14-19
    c.right = cross(up, c.direction);
    c.up = cross(c.direction, c.right);
    c.hFov = sizeH / 2.0F;  // half sizes
    c.vFov = sizeV / 2.0F;
    c.kind = 1;
    return c;
}

GCamera makePerspective(v3 position, v3 lookAt, v3 up, float hFovDeg, float vFovDeg) {
    GCamera c{};
    c.position = position;
    c.direction = normalize(lookAt - position);  // Camera.cpp:14-19
    c.right = cross(up, c.direction);
    c.up = cross(c.direction, c.right);
    c.hFov = (hFovDeg * kPi) / 180.0F;  // Camera.cpp:30-33 degToRad
    c.vFov = (vFovDeg * kPi) / 180.0F;
    c.kind = 0;
    return c;
}

GCamera cornellBoxCamera(float ratio) {
    const float fovX = 45.0F * ratio;
    return makePerspective(v3{0.0F, 0.0F, -3.4F}, v3{0.0F, 0.0F, 1.0F}, v3{0.0F, 1.0F, 0.0F}, fovX, 45.0F);
}

// ---- camera file (CameraFactory.cpp, PerspectiveLoader.cpp:18-64) ---------------------
static bool parseFloats(const std::string& s, float* out, int n) {
    std::istringstream ss(s);
    for (int i = 0; i < n; ++i) {
        float v = 0.0F;
        if (!(ss >> v)) {
            return false;
        }
        out[i] = v;
    }
    return true;
}

bool loadCameraFile(const std::string& path, float ratio, GCamera* out, std::string* err) {
    std::ifstream f(path);
    if (!f) {
        *err = "cannot open camera file " + path;
        return false;
    }
    return loadCameraStream(f, ratio, out, err, path);
}

bool loadCameraStream(std::istream& f, float ratio, GCamera* out, std::string* err, const std::string& path) {
    std::string line;
    bool perspective = false;
    while (std::getline(f, line)) {
        if (!line.empty() && line[0] == 't' && line.find("perspective") != std::string::npos) {
            perspective = true;
            break;
        }
    }
    if (!perspective) {
        *err = "camera file has no perspective camera: " + path;
        return false;
    }
    float p[3] = {0, 0, 0}, l[3] = {0, 0, 0}, u[3] = {0, 0, 0}, fov[2] = {0, 0};
    while (std::getline(f, line)) {
        if (line.empty()) continue;
        const char key = line[0];
        const std::string rest = line.substr(1);
        switch (key) {
            case 'p': parseFloats(rest, p, 3); break;
            case 'l': parseFloats(rest, l, 3); break;
            case 'u': parseFloats(rest, u, 3); break;
            case 'f': parseFloats(rest, fov, 2); break;
            default: break;
        }
    }
    p[0] = -p[0];  // PerspectiveLoader.cpp:52 "Invert X axis"
    *out = makePerspective(v3{p[0], p[1], p[2]}, v3{l[0], l[1], l[2]}, v3{u[0], u[1], u[2]}, fov[0] * ratio, fov[1]);
    return true;
}

// ---- Wavefront OBJ/MTL (tinyobjloader v1.0.7 semantics, OBJLoader.cpp) ----------------
namespace {

bool isSpace(char c) { return c == ' ' || c == '\t'; }
bool isDigit(char c) { return c >= '0' && c <= '9'; }

// tinyobjloader tryParseDouble: digits accumulated into a double mantissa, fraction digits
// added with a power-of-ten lookup table, exponent applied with ldexp/pow(5).
bool tryParseDouble(const char* s, const char* end, double* result) {
    if (s >= end) return false;
    double mantissa = 0.0;
    int exponent = 0;
    char sign = '+';
    char expSign = '+';
    const char* curr = s;
    int read = 0;
    bool endNotReached = false;
    if (*curr == '+' || *curr == '-') {
        sign = *curr;
        curr++;
    } else if (!isDigit(*curr) && *curr != '.') {
        return false;
    }
    endNotReached = (curr != end);
    while (endNotReached && isDigit(*curr)) {
        mantissa *= 10;
        mantissa += static_cast<int>(*curr - 0x30);
        curr++;
        read++;
        endNotReached = (curr != end);
    }
    if (!endNotReached) goto assemble;
    if (*curr == '.') {
        curr++;
        read = 1;
        endNotReached = (curr != end);
        while (endNotReached && isDigit(*curr)) {
            static const double powLut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            const int lutEntries = sizeof powLut / sizeof powLut[0];
            mantissa += static_cast<int>(*curr - 0x30) * (read < lutEntries ? powLut[read] : std::pow(10.0, -read));
            read++;
            curr++;
            endNotReached = (curr != end);
        }
    } else if (*curr == 'e' || *curr == 'E') {
    } else {
        goto assemble;
    }
    if (!endNotReached) goto assemble;
    if (*curr == 'e' || *curr == 'E') {
        curr++;
        endNotReached = (curr != end);
        if (endNotReached && (*curr == '+' || *curr == '-')) {
            expSign = *curr;
            curr++;
        } else if (endNotReached && isDigit(*curr)) {
        } else {
            return false;
        }
        read = 0;
        endNotReached = (curr != end);
        while (endNotReached && isDigit(*curr)) {
            exponent *= 10;
            exponent += static_cast<int>(*curr - 0x30);
            curr++;
            read++;
            endNotReached = (curr != end);
        }
        exponent *= (expSign == '+' ? 1 : -1);
        if (read == 0) return false;
    }
assemble:
    *result = (sign == '+' ? 1 : -1) *
              (exponent ? std::ldexp(mantissa * std::pow(5.0, exponent), exponent) : mantissa);
    return true;
}

// tinyobj parseReal: skip spaces, token until space/end, tryParseDouble, cast to float
float parseReal(const char** token, double def = 0.0) {
    const char* t = *token;
    while (isSpace(*t)) t++;
    const char* end = t;
    while (*end && !isSpace(*end) && *end != '\r' && *end != '\n') end++;
    double val = def;
    tryParseDouble(t, end, &val);
    *token = end;
    return static_cast<float>(val);
}

// tinyobj fixIndex: 1-based -> 0-based, negative -> relative
int fixIndex(int idx, int n) {
    if (idx > 0) return idx - 1;
    if (idx == 0) return 0;
    return n + idx;
}

struct RawMat {
    std::string name;
    float diffuse[3] = {0, 0, 0}, specular[3] = {0, 0, 0}, transmittance[3] = {0, 0, 0}, emission[3] = {0, 0, 0};
    float ior = 1.0F, dissolve = 1.0F;
    std::string diffuseTex;
};

void parseMtl(std::istream& in, std::vector<RawMat>* mats, std::unordered_map<std::string, int>* names) {
    RawMat m;
    bool hasName = false;
    bool hasD = false;
    std::string line;
    while (std::getline(in, line)) {
        while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
        const char* t = line.c_str();
        while (isSpace(*t)) t++;
        if (*t == '\0' || *t == '#') continue;
        auto key = [&t](const char* k) {
            const size_t n = std::strlen(k);
            return std::strncmp(t, k, n) == 0 && isSpace(t[n]);
        };
        auto real3 = [](const char* p, float* v) {
            v[0] = parseReal(&p);
            v[1] = parseReal(&p);
            v[2] = parseReal(&p);
        };
        if (key("newmtl")) {
            if (hasName) {
                (*names)[m.name] = static_cast<int>(mats->size());
                mats->push_back(m);
            }
            m = RawMat();
            hasD = false;
            const char* p = t + 7;
            while (isSpace(*p)) p++;
            m.name = p;
            hasName = true;
        } else if (key("Kd")) {
            real3(t + 3, m.diffuse);
        } else if (key("Ks")) {
            real3(t + 3, m.specular);
        } else if (key("Kt") || key("Tf")) {
            real3(t + 3, m.transmittance);
        } else if (key("Ke")) {
            real3(t + 3, m.emission);
        } else if (key("Ni")) {
            const char* p = t + 3;
            m.ior = parseReal(&p);
        } else if (key("d")) {
            const char* p = t + 2;
            m.dissolve = parseReal(&p);
            hasD = true;
        } else if (key("Tr")) {
            const char* p = t + 3;
            if (!hasD) m.dissolve = 1.0F - parseReal(&p);
        } else if (key("map_Kd")) {
            const char* p = t + 7;
            while (isSpace(*p)) p++;
            m.diffuseTex = p;
        }
    }
    if (hasName) {
        (*names)[m.name] = static_cast<int>(mats->size());
        mats->push_back(m);
    }
}

struct FaceIdx {
    int v, vt, vn;
};

// Utils.cpp:189-196 normalize(color)
v3 normalizeColor(v3 c) {
    const float mx = stdmax(stdmax(c.x, c.y), c.z);
    if (mx > 1.0F) return c / mx;
    return c;
}

}  // namespace

bool loadObjScene(const std::string& objPath, const std::string& mtlPath, HScene* scene, std::string* err) {
    std::ifstream mf(mtlPath);
    std::ifstream f(objPath);
    if (!f) {
        *err = "cannot open OBJ file " + objPath;
        return false;
    }
    // map_Kd textures are read from the OBJ's directory (the reference reads filePath + texname,
    // filePath being the OBJ's directory)
    const std::string objDir = objPath.find('/') == std::string::npos ? std::string() : objPath.substr(0, objPath.rfind('/') + 1);
    return loadObjStreams(f, mf ? &mf : nullptr,
                          [&objDir](const std::string& name, HTexture* tex) {
                              std::string terr;
                              return loadTextureFile(objDir + name, tex, &terr);
                          },
                          scene, err);
}

bool loadObjStreams(std::istream& f, std::istream* mtl, const TextureSource& textureSource, HScene* scene,
                    std::string* err) {
    (void)err;
    std::vector<RawMat> mats;
    std::unordered_map<std::string, int> names;
    if (mtl != nullptr) parseMtl(*mtl, &mats, &names);
    std::vector<float> vs, vns, vts, cols;
    vs.reserve(1 << 20);
    cols.reserve(1 << 20);
    struct Tri {
        FaceIdx i[3];
        int mat;
    };
    std::vector<Tri> tris;
    tris.reserve(1 << 20);
    int currentMat = -1;
    std::string line;
    std::vector<FaceIdx> face;
    while (std::getline(f, line)) {
        while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
        const char* t = line.c_str();
        while (isSpace(*t)) t++;
        if (*t == '\0' || *t == '#') continue;
        if (t[0] == 'v' && isSpace(t[1])) {
            const char* p = t + 2;
            const float x = parseReal(&p), y = parseReal(&p), z = parseReal(&p);
            // parseVertexWithColor: colours default to 1 when absent
            const float r = parseReal(&p, 1.0), g = parseReal(&p, 1.0), b = parseReal(&p, 1.0);
            vs.push_back(x);
            vs.push_back(y);
            vs.push_back(z);
            cols.push_back(r);
            cols.push_back(g);
            cols.push_back(b);
        } else if (t[0] == 'v' && t[1] == 'n' && isSpace(t[2])) {
            const char* p = t + 3;
            vns.push_back(parseReal(&p));
            vns.push_back(parseReal(&p));
            vns.push_back(parseReal(&p));
        } else if (t[0] == 'v' && t[1] == 't' && isSpace(t[2])) {
            const char* p = t + 3;
            vts.push_back(parseReal(&p));
            vts.push_back(parseReal(&p));
        } else if (t[0] == 'f' && isSpace(t[1])) {
            face.clear();
            const char* p = t + 2;
            const int nv = static_cast<int>(vs.size() / 3), nt = static_cast<int>(vts.size() / 2),
                      nn = static_cast<int>(vns.size() / 3);
            while (true) {
                while (isSpace(*p)) p++;
                if (*p == '\0') break;
                FaceIdx fi{-1, -1, -1};
                fi.v = fixIndex(std::atoi(p), nv);
                while (*p && *p != '/' && !isSpace(*p)) p++;
                if (*p == '/') {
                    p++;
                    if (*p == '/') {
                        p++;
                        fi.vn = fixIndex(std::atoi(p), nn);
                        while (*p && !isSpace(*p)) p++;
                    } else {
                        fi.vt = fixIndex(std::atoi(p), nt);
                        while (*p && *p != '/' && !isSpace(*p)) p++;
                        if (*p == '/') {
                            p++;
                            fi.vn = fixIndex(std::atoi(p), nn);
                            while (*p && !isSpace(*p)) p++;
                        }
                    }
                }
                face.push_back(fi);
            }
            // tinyobjloader v1.0.7 triangulation: fan around the first vertex
            for (size_t k = 2; k < face.size(); ++k) {
                tris.push_back(Tri{{face[0], face[k - 1], face[k]}, currentMat});
            }
        } else if (std::strncmp(t, "usemtl", 6) == 0 && isSpace(t[6])) {
            const char* p = t + 7;
            while (isSpace(*p)) p++;
            std::string name(p);
            while (!name.empty() && isSpace(name.back())) name.pop_back();
            auto it = names.find(name);
            currentMat = (it == names.end()) ? -1 : it->second;
        }
    }

    // map_Kd textures, loaded once per file name (OBJLoader.cpp:224-242)
    std::unordered_map<std::string, int32_t> texCache;
    auto textureOf = [&](const std::string& name) -> int32_t {
        auto it = texCache.find(name);
        if (it != texCache.end()) return it->second;
        HTexture tex;
        int32_t id = -1;
        if (textureSource(name, &tex)) {  // Texture::isValid (Texture.cpp:137-139)
            id = static_cast<int32_t>(scene->textures.size());
            scene->textures.push_back(std::move(tex));
        }
        texCache[name] = id;
        return id;
    };
    auto fract = [](float x) { return x - std::floor(x); };  // glm::fract (Utils.cpp:177-180)
    const bool hasNormals = !vns.empty();
    auto vert = [&vs](int i) { return v3{-vs[3 * i], vs[3 * i + 1], vs[3 * i + 2]}; };  // OBJLoader.cpp:139-141
    auto nrm = [&vns](int i) { return v3{-vns[3 * i], vns[3 * i + 1], vns[3 * i + 2]}; }; // :170-172
    const v2 noTex{-1.0F, -1.0F};
    scene->triangles.reserve(scene->triangles.size() + tris.size());
    for (const Tri& tr : tris) {
        const v3 a = vert(tr.i[0].v), b = vert(tr.i[1].v), c = vert(tr.i[2].v);
        v3 na, nb, nc;
        if (hasNormals && tr.i[0].vn >= 0 && tr.i[1].vn >= 0 && tr.i[2].vn >= 0) {
            na = nrm(tr.i[0].vn);
            nb = nrm(tr.i[1].vn);
            nc = nrm(tr.i[2].vn);
        } else {
            const v3 ab = b - a, ac = c - a;
            na = nb = nc = normalize(cross(ac, ab));  // OBJLoader.cpp:176-182
        }
        HMaterial m;
        v2 texA = noTex, texB = noTex, texC = noTex;
        if (tr.mat >= 0) {
            const RawMat& rm = mats[static_cast<size_t>(tr.mat)];
            m.Kd = v3{rm.diffuse[0], rm.diffuse[1], rm.diffuse[2]};
            m.Ks = v3{rm.specular[0], rm.specular[1], rm.specular[2]};
            m.Kt = v3{rm.transmittance[0], rm.transmittance[1], rm.transmittance[2]} * (1.0F - rm.dissolve);
            m.Le = normalizeColor(v3{rm.emission[0], rm.emission[1], rm.emission[2]});
            m.ior = rm.ior;
            // OBJLoader.cpp:332-364: a texture and texture coordinates -> the texture and the
            // corners' coordinates wrapped into [0, 1); an invalid texture -> coordinates -1
            if (!rm.diffuseTex.empty() && !vts.empty()) {
                m.texture = rm.diffuseTex;
                m.texId = textureOf(rm.diffuseTex);
                if (m.texId < 0) m.texture = "";  // unreadable: the reference would throw (Texture.cpp:88-92)
                bool allVt = true;
                for (int k = 0; k < 3; ++k) allVt = allVt && tr.i[k].vt >= 0;
                if (m.texId >= 0 && allVt) {
                    v2 tc[3];
                    for (int k = 0; k < 3; ++k) {
                        const int t = tr.i[k].vt;
                        tc[k] = v2{fract(vts[2 * static_cast<size_t>(t)]), fract(vts[2 * static_cast<size_t>(t) + 1])};
                    }
                    texA = tc[0];
                    texB = tc[1];
                    texC = tc[2];
                }
            }
        } else {
            const int vi = tr.i[0].v;  // OBJLoader.cpp:423-433 vertex colour of the first vertex
            m.Kd = v3{cols[3 * vi], cols[3 * vi + 1], cols[3 * vi + 2]};
        }
        if (tr.mat >= 0 && hasPositive(m.Le)) {
            HLight l;
            l.kind = kAreaLight;
            l.radiance = m;
            l.position = v3{0, 0, 0};
            l.tri = makeTriangle(a, b, c, na, nb, nc, noTex, noTex, noTex, -1);
            scene->lights.push_back(l);
            continue;
        }
        int32_t matIndex = -1;
        for (size_t k = 0; k < scene->materials.size(); ++k) {  // OBJLoader.cpp:406-418
            if (materialEqual(scene->materials[k], m)) {
                matIndex = static_cast<int32_t>(k);
                break;
            }
        }
        if (matIndex < 0) {
            matIndex = static_cast<int32_t>(scene->materials.size());
            scene->materials.push_back(m);
        }
        scene->triangles.push_back(makeTriangle(a, b, c, na, nb, nc, texA, texB, texC, matIndex));
    }
    return true;
}

// ---- BVH build (BVH.hpp:126-283, 398-460) ------------------------------------------------
namespace {

float surfaceArea(const HAABB& b) {  // AABB.cpp:61-71
    const v3 l = b.mx - b.mn;
    const float bottomTop = 2.0F * l.x * l.z;
    const float sideXY = 2.0F * l.x * l.y;
    const float sideZY = 2.0F * l.z * l.y;
    return bottomTop + sideXY + sideZY;
}

v3 centroid(const HAABB& b) {  // AABB.cpp:81-85
    const v3 len = (b.mx - b.mn) / 2.0F;
    return b.mn + len;
}

HAABB surrounding(const HAABB& a, const HAABB& b) { return HAABB{vmin(a.mn, b.mn), vmax(a.mx, b.mx)}; }

int32_t splitIndexSah(const std::vector<HAABB>& boxes) {  // BVH.hpp:398-439
    const long numberBoxes = static_cast<long>(boxes.size());
    const long numBoxes = numberBoxes - 1;
    std::vector<float> leftArea(static_cast<size_t>(numBoxes));
    HAABB leftBox = boxes[0];
    leftArea[0] = surfaceArea(leftBox);
    for (long i = 1; i < numBoxes; ++i) {
        leftBox = surrounding(leftBox, boxes[static_cast<size_t>(i)]);
        leftArea[static_cast<size_t>(i)] = surfaceArea(leftBox);
    }
    std::vector<float> rightArea(static_cast<size_t>(numBoxes));
    HAABB rightBox = boxes[static_cast<size_t>(numBoxes)];
    rightArea[static_cast<size_t>(numBoxes - 1)] = surfaceArea(rightBox);
    for (long i = numBoxes - 2; i >= 0; --i) {
        rightBox = surrounding(rightBox, boxes[static_cast<size_t>(i + 1)]);
        rightArea[static_cast<size_t>(i)] = surfaceArea(rightBox);
    }
    int32_t splitIndex = 1;
    float minSah = leftArea[0] + static_cast<float>(numBoxes) * rightArea[0];
    for (long i = 1; i < numBoxes; ++i) {
        const long nL = i + 1;
        const long nR = numberBoxes - nL;
        const float sah = static_cast<float>(nL) * leftArea[static_cast<size_t>(i)] +
                          static_cast<float>(nR) * rightArea[static_cast<size_t>(i)];
        if (sah < minSah) {
            splitIndex = static_cast<int32_t>(i + 1);
            minSah = sah;
        }
    }
    return splitIndex;
}

struct BuildNode {
    HAABB box;
    v3 c;
    int32_t oldIndex;
};

}  // namespace

// One node of the build (BVH.hpp:161-283 loop body): bucket partition of bn[begin, end) along
// the longest axis, the node box, then leaf (<= 4 prims) or SAH split.  Children go to slots
// freeBase and freeBase + 1; a subtree of m prims owns 2m - 1 slots (its root's slot plus
// 2m - 2 for descendants), so disjoint subtrees can be built concurrently and every node's
// partition - hence the primitive order and every box - is the serial build's.
struct BuildTask {
    int32_t slot, begin, end, freeBase;
};

static int processNode(std::vector<BuildNode>& bn, std::vector<HBVHNode>& nodes, const BuildTask& t,
                       std::vector<HAABB>& boxes, BuildTask* children) {
    const int32_t begin = t.begin, end = t.end;
    // getSurroundingBox (BVH.hpp:451-460)
    HAABB sur{bn[static_cast<size_t>(begin)].box.mn, bn[static_cast<size_t>(begin)].box.mx};
    for (int32_t i = begin + 1; i < end; ++i) sur = surrounding(sur, bn[static_cast<size_t>(i)].box);
    const v3 maxDist = sur.mx - sur.mn;
    const int axis = (maxDist.x >= maxDist.y && maxDist.x >= maxDist.z)
                         ? 0
                         : ((maxDist.y >= maxDist.x && maxDist.y >= maxDist.z) ? 1 : 2);
    const int numBuckets = 10;
    const v3 step = maxDist / static_cast<float>(numBuckets);
    const float stepAxis = comp(step, axis);
    const float startBox = comp(sur.mn, axis);
    const float limit1 = startBox + stepAxis;
    auto first = bn.begin() + begin;
    auto last = bn.begin() + end;
    auto itBucket = pinnedPartition(first, last, [axis, limit1](const BuildNode& x) { return comp(x.c, axis) < limit1; });
    for (int32_t bi = 2; bi < numBuckets; ++bi) {
        const float limit = startBox + stepAxis * static_cast<float>(bi);
        itBucket = pinnedPartition(itBucket, last, [axis, limit](const BuildNode& x) { return comp(x.c, axis) < limit; });
    }
    HBVHNode& node = nodes[static_cast<size_t>(t.slot)];
    node.box = bn[static_cast<size_t>(begin)].box;
    boxes.clear();
    boxes.push_back(node.box);
    for (int32_t i = begin + 1; i < end; ++i) {
        const HAABB nb = bn[static_cast<size_t>(i)].box;
        node.box = surrounding(nb, node.box);
        boxes.push_back(nb);
    }
    const int32_t count = end - begin;
    if (count <= 4) {  // maxPrimitivesInBoxLeaf (BVH.hpp:239-251)
        node.indexOffset = begin;
        node.numPrimitives = count;
        return 0;
    }
    const int32_t split = splitIndexSah(boxes);
    node.indexOffset = t.freeBase;
    node.numPrimitives = 0;
    const int32_t leftFree = t.freeBase + 2;
    children[0] = BuildTask{t.freeBase, begin, begin + split, leftFree};
    children[1] = BuildTask{t.freeBase + 1, begin + split, end, leftFree + 2 * split - 2};
    return 2;
}

template <class T>
std::vector<HBVHNode> buildBVH(std::vector<T>* primsPtr, std::vector<int32_t>* order) {
    std::vector<T>& prims = *primsPtr;
    std::vector<HBVHNode> nodes;
    order->clear();
    if (prims.empty()) {
        nodes.push_back(HBVHNode{HAABB{v3{0, 0, 0}, v3{0, 0, 0}}, 0, 0});
        return nodes;
    }
    const int32_t n = static_cast<int32_t>(prims.size());
    nodes.assign(static_cast<size_t>(2 * n - 1), HBVHNode{HAABB{v3{0, 0, 0}, v3{0, 0, 0}}, 0, 0});
    std::vector<BuildNode> bn;
    bn.reserve(prims.size());
    for (int32_t i = 0; i < n; ++i) {
        const HAABB b = aabbOf(prims[static_cast<size_t>(i)]);
        bn.push_back(BuildNode{b, centroid(b), i});
    }
    // the top of the tree level by level (the nodes of a level in parallel) until there are
    // enough subtrees ...
    const int workers = static_cast<int>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
    constexpr int32_t kSerialBelow = 2048;  // subtrees smaller than this are not worth a hand-off
    std::vector<BuildTask> frontier{BuildTask{0, 0, n, 1}};
    std::vector<BuildTask> subtrees;
    while (!frontier.empty() && static_cast<int>(frontier.size() + subtrees.size()) < 8 * workers) {
        std::vector<BuildTask> level;
        for (const BuildTask& t : frontier) {
            if (workers == 1 || t.end - t.begin < kSerialBelow) {
                subtrees.push_back(t);
            } else {
                level.push_back(t);
            }
        }
        std::vector<BuildTask> kids(2 * level.size());
        std::vector<int> nk(level.size(), 0);
        std::vector<std::thread> lt;
        for (size_t i = 0; i < level.size(); ++i) {
            lt.emplace_back([&, i]() {
                std::vector<HAABB> scratch;
                nk[i] = processNode(bn, nodes, level[i], scratch, &kids[2 * i]);
            });
        }
        for (auto& th : lt) th.join();
        frontier.clear();
        for (size_t i = 0; i < level.size(); ++i)
            for (int c = 0; c < nk[i]; ++c) frontier.push_back(kids[2 * i + static_cast<size_t>(c)]);
    }
    subtrees.insert(subtrees.end(), frontier.begin(), frontier.end());
    std::sort(subtrees.begin(), subtrees.end(),
              [](const BuildTask& x, const BuildTask& y) { return x.end - x.begin > y.end - y.begin; });
    // ... then the subtrees depth-first, largest first, on a pool of threads
    std::atomic<size_t> next{0};
    auto worker = [&]() {
        std::vector<HAABB> scratch;
        std::vector<BuildTask> stack;
        BuildTask kids[2];
        for (size_t i = next.fetch_add(1); i < subtrees.size(); i = next.fetch_add(1)) {
            stack.assign(1, subtrees[i]);
            while (!stack.empty()) {
                const BuildTask t = stack.back();
                stack.pop_back();
                const int k = processNode(bn, nodes, t, scratch, kids);
                if (k == 2) {  // left first (the serial order; results do not depend on it)
                    stack.push_back(kids[1]);
                    stack.push_back(kids[0]);
                }
            }
        }
    };
    std::vector<std::thread> pool;
    const int spawn = std::min<int>(workers, static_cast<int>(subtrees.size())) - 1;
    for (int w = 0; w < spawn; ++w) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    std::vector<T> permuted;
    permuted.reserve(prims.size());
    order->reserve(prims.size());
    for (int32_t i = 0; i < n; ++i) {
        const int32_t old = bn[static_cast<size_t>(i)].oldIndex;
        permuted.push_back(prims[static_cast<size_t>(old)]);
        order->push_back(old);
    }
    prims.swap(permuted);
    return nodes;
}

template std::vector<HBVHNode> buildBVH<HTriangle>(std::vector<HTriangle>*, std::vector<int32_t>*);
template std::vector<HBVHNode> buildBVH<HPlane>(std::vector<HPlane>*, std::vector<int32_t>*);
template std::vector<HBVHNode> buildBVH<HSphere>(std::vector<HSphere>*, std::vector<int32_t>*);

// Device BVH2: one GNode per inner node, holding both children's boxes.  Inner nodes are
// renumbered: the first topCount in breadth-first order (the levels every ray crosses; the
// trace kernels can stage them in LDS), the rest in depth-first pre-order, left child first,
// so a parent and its left child usually share a 128-byte line.  Node numbering does not
// affect results (boxes, child order and leaves are the reference's).
void toDeviceBVH(const std::vector<HBVHNode>& nodes, size_t numPrims, std::vector<GNode>* out, GRoot* root,
                 int topCount, int* topPlaced, const std::vector<uint32_t>* cones) {
    out->clear();
    if (topPlaced != nullptr) *topPlaced = 0;
    const HBVHNode& r = nodes[0];
    root->bmin[0] = r.box.mn.x;
    root->bmin[1] = r.box.mn.y;
    root->bmin[2] = r.box.mn.z;
    root->bmax[0] = r.box.mx.x;
    root->bmax[1] = r.box.mx.y;
    root->bmax[2] = r.box.mx.z;
    root->count = static_cast<int32_t>(numPrims);
    if (numPrims == 0) {
        root->ref = 0;
        return;
    }
    if (r.numPrimitives > 0) {
        root->ref = leafRef(r.indexOffset, r.numPrimitives);
        return;
    }
    auto inner = [&](int32_t i) { return nodes[static_cast<size_t>(i)].numPrimitives == 0; };
    std::vector<int32_t> newIdx(nodes.size(), -1);
    std::vector<int32_t> order;
    std::deque<int32_t> bfs{0};
    while (!bfs.empty() && static_cast<int>(order.size()) < topCount) {
        const int32_t i = bfs.front();
        bfs.pop_front();
        newIdx[static_cast<size_t>(i)] = static_cast<int32_t>(order.size());
        order.push_back(i);
        const int32_t l = nodes[static_cast<size_t>(i)].indexOffset;
        if (inner(l)) bfs.push_back(l);
        if (inner(l + 1)) bfs.push_back(l + 1);
    }
    if (topPlaced != nullptr) *topPlaced = static_cast<int>(order.size());
    auto place = [&](int32_t i) {
        newIdx[static_cast<size_t>(i)] = static_cast<int32_t>(order.size());
        order.push_back(i);
    };
    std::vector<int32_t> dfs{0};
    while (!dfs.empty()) {
        const int32_t i = dfs.back();
        dfs.pop_back();
        if (newIdx[static_cast<size_t>(i)] < 0) place(i);
        const int32_t l = nodes[static_cast<size_t>(i)].indexOffset;
        if (inner(l + 1)) dfs.push_back(l + 1);
        if (inner(l)) dfs.push_back(l);
    }
    auto ref = [&](int32_t j) {
        const HBVHNode& c = nodes[static_cast<size_t>(j)];
        return c.numPrimitives > 0 ? leafRef(c.indexOffset, c.numPrimitives) : newIdx[static_cast<size_t>(j)];
    };
    root->ref = 0;
    out->resize(order.size());
    for (size_t k = 0; k < order.size(); ++k) {
        const int32_t l = nodes[static_cast<size_t>(order[k])].indexOffset;
        const HBVHNode& L = nodes[static_cast<size_t>(l)];
        const HBVHNode& R = nodes[static_cast<size_t>(l + 1)];
        GNode g{};
        g.lminx = L.box.mn.x;
        g.lminy = L.box.mn.y;
        g.lminz = L.box.mn.z;
        g.lmaxx = L.box.mx.x;
        g.lmaxy = L.box.mx.y;
        g.lmaxz = L.box.mx.z;
        g.rminx = R.box.mn.x;
        g.rminy = R.box.mn.y;
        g.rminz = R.box.mn.z;
        g.rmaxx = R.box.mx.x;
        g.rmaxy = R.box.mx.y;
        g.rmaxz = R.box.mx.z;
        g.refL = ref(l);
        g.refR = ref(l + 1);
        g.coneL = cones != nullptr ? (*cones)[static_cast<size_t>(l)] : kConeNever;
        g.coneR = cones != nullptr ? (*cones)[static_cast<size_t>(l + 1)] : kConeNever;
        (*out)[k] = g;
    }
}

// Outward 16-bit quantization of the walk tree.  The kernel evaluates a
// plane as t = fma(q, fl(step * inv), fl(fl(origin - o) * inv)); for a ray whose origin lies
// within 4 grid extents of the origin and whose 1/d components are in [2^-40, 2^90] that value is
// within S |1/d| 2^-19 (S = the grid extent on that axis) of (origin + q step - o) / d, and the
// reference's (b - o) * inv of an exact box b within as much of (b - o) / d.  A margin of one
// grid step (S / 65535 > S 2^-19) on each side therefore keeps every computed slab interval of a
// node around the computed interval of every reference leaf box below it.
namespace {
// the walk tree's grid over a root box, and the outward rounding of one coordinate
struct Quantizer {
    double step[3] = {}, org[3] = {};
    bool init(const float* bmin, const float* bmax, QGrid* grid) {
        double lo[3], ext[3], emax = 0.0;
        for (int a = 0; a < 3; ++a) {
            lo[a] = bmin[a];
            ext[a] = static_cast<double>(bmax[a]) - bmin[a];
            if (!std::isfinite(lo[a]) || !std::isfinite(ext[a]) || ext[a] < 0.0) return false;
            emax = std::max(emax, ext[a]);
        }
        for (int a = 0; a < 3; ++a) {
            const double e = std::max({ext[a], emax * 0x1p-10, 0x1p-20});
            // 65535 steps from origin = min - 2 step must reach max + 2 step: step >= e / 65531
            const float sf = std::nextafter(static_cast<float>(e / 65528.0), std::numeric_limits<float>::infinity());
            const float of = std::nextafter(static_cast<float>(lo[a] - 2.0 * sf), -std::numeric_limits<float>::infinity());
            if (!std::isfinite(sf) || !std::isfinite(of) || !(sf > 0.0F)) return false;
            step[a] = sf;
            org[a] = of;
            grid->step[a] = sf;
            grid->origin[a] = of;
        }
        return true;
    }
    uint32_t lo(float b, int a) const {  // largest q with origin + q step <= b - step
        double q = std::floor((static_cast<double>(b) - org[a]) / step[a]) - 1.0;
        q = std::min(std::max(q, 0.0), 65535.0);
        while (q > 0.0 && org[a] + q * step[a] > static_cast<double>(b) - step[a]) q -= 1.0;
        return static_cast<uint32_t>(q);
    }
    uint32_t hi(float b, int a) const {  // smallest q with origin + q step >= b + step
        double q = std::ceil((static_cast<double>(b) - org[a]) / step[a]) + 1.0;
        q = std::min(std::max(q, 0.0), 65535.0);
        while (q < 65535.0 && org[a] + q * step[a] < static_cast<double>(b) + step[a]) q += 1.0;
        return static_cast<uint32_t>(q);
    }
    // one box as three words, one per axis: min | max << 16 (the walk rotates a word by 16 bits
    // when the ray's 1/d is negative on that axis, mrt_trace_ww.hpp qslabNF, so min <= max)
    bool box(const float* mn, const float* mx, uint32_t* w) const {
        for (int a = 0; a < 3; ++a)
            if (!std::isfinite(mn[a]) || !std::isfinite(mx[a])) return false;
        for (int a = 0; a < 3; ++a) {
            const uint32_t l = lo(mn[a], a), h = hi(mx[a], a);
            if (l > h) return false;
            w[a] = l | (h << 16);
        }
        return true;
    }
};
}  // namespace

// The optimal collapse's dynamic programme (toQuantizedBVH4): forest[i * (W + 1) + j] = the least
// summed wide-node area covering BVH2 node i's subtree with at most j trees, split[] its choices.
// forest[1] (the root as a wide node) is the whole wide tree's cost.
static void collapseForests(const std::vector<HBVHNode>& nodes, std::vector<double>* forestOut,
                            std::vector<int8_t>* splitOut, const std::vector<double>* nodeCost = nullptr) {
    auto inner = [&](int32_t i) { return nodes[static_cast<size_t>(i)].numPrimitives == 0; };
    auto area = [&](int32_t i) {
        if (nodeCost != nullptr) return (*nodeCost)[static_cast<size_t>(i)];
        const HAABB& b = nodes[static_cast<size_t>(i)].box;
        const double dx = static_cast<double>(b.mx.x) - b.mn.x, dy = static_cast<double>(b.mx.y) - b.mn.y,
                     dz = static_cast<double>(b.mx.z) - b.mn.z;
        return dx * dy + dy * dz + dz * dx;
    };
    constexpr int W1 = kWalkWidth + 1;
    std::vector<double>& forest = *forestOut;
    std::vector<int8_t>& split = *splitOut;
    {
        forest.assign(nodes.size() * W1, 0.0);  // leaves: 0 (the same in every tree)
        split.assign(nodes.size() * W1, 0);
        std::vector<std::pair<int32_t, bool>> post{{0, false}};
        while (!post.empty()) {
            const auto [i, done] = post.back();
            post.pop_back();
            if (!inner(i)) continue;
            const size_t ui = static_cast<size_t>(i);
            const int32_t l = nodes[ui].indexOffset, r = l + 1;
            if (!done) {
                post.push_back({i, true});
                post.push_back({l, false});
                post.push_back({r, false});
                continue;
            }
            const size_t ul = static_cast<size_t>(l) * W1, ur = static_cast<size_t>(r) * W1;
            auto best = [&](int j, int* k) {  // at most j trees split between the two children
                double c = std::numeric_limits<double>::infinity();
                for (int a = 1; a < j; ++a) {
                    const double v = forest[ul + static_cast<size_t>(a)] + forest[ur + static_cast<size_t>(j - a)];
                    if (v < c) {
                        c = v;
                        *k = a;
                    }
                }
                return c;
            };
            int kw = 1;
            const double asWide = area(i) + best(kWalkWidth, &kw);  // node i as a wide node
            split[ui * W1] = static_cast<int8_t>(kw);
            forest[ui * W1 + 1] = asWide;
            for (int j = 2; j < W1; ++j) {
                int k = 1;
                const double c = best(j, &k);
                const bool self = asWide <= c;
                forest[ui * W1 + static_cast<size_t>(j)] = self ? asWide : c;
                split[ui * W1 + static_cast<size_t>(j)] = static_cast<int8_t>(self ? 0 : k);
            }
        }
    }
}

// The optimal collapse's summed wide-node area and its depth in wide nodes (0 without an inner node)
static double collapsedArea(const std::vector<HBVHNode>& nodes, int* depth) {
    *depth = 0;
    if (nodes.size() < 3 || nodes[0].numPrimitives > 0) return 0.0;  // no inner node (an empty scene: one empty root)
    std::vector<double> forest;
    std::vector<int8_t> split;
    collapseForests(nodes, &forest, &split);
    constexpr int W1 = kWalkWidth + 1;
    auto inner = [&](int32_t i) { return nodes[static_cast<size_t>(i)].numPrimitives == 0; };
    // the wide nodes as toQuantizedBVH4 forms them: node i's children are the trees of the best
    // forests under its two BVH2 children; an inner tree root is a wide node one level down
    std::function<void(int32_t, int, std::vector<int32_t>&)> trees = [&](int32_t i, int j, std::vector<int32_t>& out) {
        const int k = inner(i) && j > 1 ? split[static_cast<size_t>(i) * W1 + static_cast<size_t>(j)] : 0;
        if (k == 0) {
            out.push_back(i);
            return;
        }
        trees(nodes[static_cast<size_t>(i)].indexOffset, k, out);
        trees(nodes[static_cast<size_t>(i)].indexOffset + 1, j - k, out);
    };
    std::vector<std::pair<int32_t, int>> st{{0, 1}};
    while (!st.empty()) {
        const auto [i, d] = st.back();
        st.pop_back();
        *depth = std::max(*depth, d);
        const int32_t l = nodes[static_cast<size_t>(i)].indexOffset;
        const int kw = split[static_cast<size_t>(i) * W1];
        std::vector<int32_t> c;
        trees(l, kw, c);
        trees(l + 1, kWalkWidth - kw, c);
        for (const int32_t k : c)
            if (inner(k)) st.push_back({k, d + 1});
    }
    return forest[1];
}

bool toQuantizedBVH4(const std::vector<HBVHNode>& nodes, size_t numPrims, GRoot* root, int topCount, int* topPlaced,
                     QGrid* grid, std::vector<QNode4>* out, std::vector<int32_t>* bvh2Of,
                     const std::vector<double>* nodeCost) {
    out->clear();
    if (bvh2Of != nullptr) bvh2Of->clear();
    if (topPlaced != nullptr) *topPlaced = 0;
    const HBVHNode& r = nodes[0];
    const float rmn[3] = {r.box.mn.x, r.box.mn.y, r.box.mn.z}, rmx[3] = {r.box.mx.x, r.box.mx.y, r.box.mx.z};
    for (int a = 0; a < 3; ++a) {
        root->bmin[a] = rmn[a];
        root->bmax[a] = rmx[a];
    }
    root->count = static_cast<int32_t>(numPrims);
    root->ref = 0;
    Quantizer qz;
    const bool gridOK = qz.init(rmn, rmx, grid);
    if (numPrims == 0) return gridOK;
    if (r.numPrimitives > 0) {
        root->ref = leafRef(r.indexOffset, r.numPrimitives);
        return gridOK;
    }
    if (!gridOK) return false;
    auto inner = [&](int32_t i) { return nodes[static_cast<size_t>(i)].numPrimitives == 0; };
    auto area = [&](int32_t i) {
        const HAABB& b = nodes[static_cast<size_t>(i)].box;
        const double dx = static_cast<double>(b.mx.x) - b.mn.x, dy = static_cast<double>(b.mx.y) - b.mn.y,
                     dz = static_cast<double>(b.mx.z) - b.mn.z;
        return dx * dy + dy * dz + dz * dx;
    };
    // Optimal collapse (MOBILERT_COLLAPSE != "greedy"): the walk visits every wide node whose box
    // the ray passes (no inner node is culled in the exact mode), each visit testing all its
    // children, so the expected cost of a wide tree is proportional to the summed surface area of
    // its wide nodes (the leaves are the same in every collapse).  Dynamic programming over the
    // BVH2 (Ylitie et al. 2017): forest[i][j] = the least cost of covering node i's subtree with at
    // most j trees, each tree root a leaf or a wide node; a wide node's children are the best
    // forest of at most kWalkWidth trees under its two BVH2 children.
    const char* collapseEnv = std::getenv("MOBILERT_COLLAPSE");
    const bool optimal = collapseEnv == nullptr || std::string(collapseEnv) != "greedy";
    constexpr int W1 = kWalkWidth + 1;
    std::vector<double> forest;  // [i * W1 + j], j = 1..kWalkWidth
    std::vector<int8_t> split;   // [i * W1 + j]: trees taken from the left child (0: node i itself);
                                 // [i * W1]: the split of node i as a wide node
    if (optimal) collapseForests(nodes, &forest, &split, nodeCost);
    // the trees of node i's best forest of at most j (BVH2 indices, left to right)
    std::function<void(int32_t, int, std::vector<int32_t>&)> trees = [&](int32_t i, int j, std::vector<int32_t>& out) {
        const int k = inner(i) && j > 1 ? split[static_cast<size_t>(i) * W1 + static_cast<size_t>(j)] : 0;
        if (k == 0) {
            out.push_back(i);
            return;
        }
        trees(nodes[static_cast<size_t>(i)].indexOffset, k, out);
        trees(nodes[static_cast<size_t>(i)].indexOffset + 1, j - k, out);
    };
    // collapse: the 4-wide node of BVH2 node i has up to four BVH2 descendants as children
    std::vector<std::array<int32_t, kWalkWidth>> kids;  // per walk node: BVH2 indices (-1: none)
    std::vector<int32_t> node4Of(nodes.size(), -1);
    std::vector<int32_t> kidsBvh2{0};  // per walk node: its BVH2 node
    std::vector<int32_t> work{0};
    node4Of[0] = 0;
    kids.emplace_back();
    kids.back().fill(-1);
    while (!work.empty()) {
        const int32_t i = work.back();
        work.pop_back();
        const int32_t l = nodes[static_cast<size_t>(i)].indexOffset;
        std::vector<int32_t> c{l, l + 1};
        if (optimal) {  // node i's best split into at most kWalkWidth trees
            const int kw = split[static_cast<size_t>(i) * W1];
            c.clear();
            trees(l, kw, c);
            trees(l + 1, kWalkWidth - kw, c);
        }
        while (!optimal && c.size() < static_cast<size_t>(kWalkWidth)) {
            int best = -1;
            double ba = -1.0;
            for (size_t k = 0; k < c.size(); ++k)
                if (inner(c[k]) && area(c[k]) > ba) {
                    ba = area(c[k]);
                    best = static_cast<int>(k);
                }
            if (best < 0) break;
            const int32_t cl = nodes[static_cast<size_t>(c[static_cast<size_t>(best)])].indexOffset;
            c[static_cast<size_t>(best)] = cl;
            c.insert(c.begin() + best + 1, cl + 1);
        }
        std::array<int32_t, kWalkWidth> k4;
        k4.fill(-1);
        for (size_t k = 0; k < c.size(); ++k) {
            k4[k] = c[k];
            if (inner(c[k])) {
                node4Of[static_cast<size_t>(c[k])] = static_cast<int32_t>(kids.size());
                kidsBvh2.push_back(c[k]);
                kids.emplace_back();
                kids.back().fill(-1);
                work.push_back(c[k]);
            }
        }
        kids[static_cast<size_t>(node4Of[static_cast<size_t>(i)])] = k4;
    }
    // numbering: the first topCount breadth-first, the rest depth-first pre-order
    const size_t n4 = kids.size();
    std::vector<int32_t> newIdx(n4, -1), order;
    std::deque<int32_t> bfs{0};
    while (!bfs.empty() && static_cast<int>(order.size()) < topCount) {
        const int32_t j = bfs.front();
        bfs.pop_front();
        newIdx[static_cast<size_t>(j)] = static_cast<int32_t>(order.size());
        order.push_back(j);
        for (int32_t c : kids[static_cast<size_t>(j)])
            if (c >= 0 && inner(c)) bfs.push_back(node4Of[static_cast<size_t>(c)]);
    }
    if (topPlaced != nullptr) *topPlaced = static_cast<int>(order.size());
    std::vector<int32_t> dfs{0};
    while (!dfs.empty()) {
        const int32_t j = dfs.back();
        dfs.pop_back();
        if (newIdx[static_cast<size_t>(j)] < 0) {
            newIdx[static_cast<size_t>(j)] = static_cast<int32_t>(order.size());
            order.push_back(j);
        }
        const auto& k4 = kids[static_cast<size_t>(j)];
        for (int k = kWalkWidth - 1; k >= 0; --k)
            if (k4[static_cast<size_t>(k)] >= 0 && inner(k4[static_cast<size_t>(k)]))
                dfs.push_back(node4Of[static_cast<size_t>(k4[static_cast<size_t>(k)])]);
    }
    out->resize(n4);
    if (bvh2Of != nullptr) {
        bvh2Of->resize(n4);
        for (size_t k = 0; k < n4; ++k) (*bvh2Of)[k] = kidsBvh2[static_cast<size_t>(order[k])];
    }
    for (size_t k = 0; k < n4; ++k) {
        const auto& k4 = kids[static_cast<size_t>(order[k])];
        QNode4& q = (*out)[k];
        for (int c = 0; c < kWalkWidth; ++c) {
            const int32_t b = k4[static_cast<size_t>(c)];
            if (b < 0) {
                // an inverted box (min 65535, max 0 on every axis): the per-lane walk's near / far
                // test (qslabNF) misses it for every quantOK ray, so it needs no slot check
                q.q[3 * c] = q.q[3 * c + 1] = q.q[3 * c + 2] = 0xFFFFu;
                q.ref[c] = kEmptyChild;
                continue;
            }
            const HBVHNode& bn = nodes[static_cast<size_t>(b)];
            const float mn[3] = {bn.box.mn.x, bn.box.mn.y, bn.box.mn.z}, mx[3] = {bn.box.mx.x, bn.box.mx.y, bn.box.mx.z};
            if (!qz.box(mn, mx, q.q + 3 * c)) {
                out->clear();
                return false;
            }
            q.ref[c] = bn.numPrimitives > 0 ? leafRef(bn.indexOffset, bn.numPrimitives)
                                             : newIdx[static_cast<size_t>(node4Of[static_cast<size_t>(b)])];
        }
    }
    root->ref = 0;
    return true;
}

namespace {
// one node's cull word from its triangles [lo, hi) (BVH order)
uint32_t coneWord(const std::vector<HTriangle>& tris, size_t lo, size_t hi) {
    // K: conditioning of Moller-Trumbore's determinant (Triangle.cpp:67-70) for every triangle
    double kMax = 1.0;
    double m[3][3] = {};  // sum of n n^T over unit normals (sign-free: lines, not directions)
    std::vector<std::array<double, 3>> ns;
    ns.reserve(hi - lo);
    for (size_t i = lo; i < hi; ++i) {
        const HTriangle& t = tris[i];
        const double ab[3] = {t.AB.x, t.AB.y, t.AB.z}, ac[3] = {t.AC.x, t.AC.y, t.AC.z};
        const double n[3] = {ab[1] * ac[2] - ab[2] * ac[1], ab[2] * ac[0] - ab[0] * ac[2], ab[0] * ac[1] - ab[1] * ac[0]};
        const double len = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        const double l1 = (std::fabs(ab[0]) + std::fabs(ab[1]) + std::fabs(ab[2])) *
                          (std::fabs(ac[0]) + std::fabs(ac[1]) + std::fabs(ac[2]));
        if (!(len > 0.0) || !std::isfinite(l1)) return kConeNever;  // degenerate: no bound
        kMax = std::max(kMax, l1 / len);
        const std::array<double, 3> u{n[0] / len, n[1] / len, n[2] / len};
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) m[r][c] += u[static_cast<size_t>(r)] * u[static_cast<size_t>(c)];
        ns.push_back(u);
    }
    const double kCode = std::ceil(8.0 * std::log2(kMax) + 1e-9);
    if (ns.empty() || kCode > 126.0) return kConeNever;
    // axis: dominant eigenvector of sum n n^T (power iteration from the largest column)
    int col = 0;
    for (int c = 1; c < 3; ++c)
        if (m[c][c] > m[col][col]) col = c;
    double a[3] = {m[0][col], m[1][col], m[2][col]};
    for (int it = 0; it < 64; ++it) {
        double b[3];
        for (int r = 0; r < 3; ++r) b[r] = m[r][0] * a[0] + m[r][1] * a[1] + m[r][2] * a[2];
        const double l = std::sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
        if (!(l > 0.0)) return kConeNever;
        for (int r = 0; r < 3; ++r) a[r] = b[r] / l;
    }
    // octahedral encoding of a, then the cone around the DECODED axis (as the kernel sees it)
    const double s1 = std::fabs(a[0]) + std::fabs(a[1]) + std::fabs(a[2]);
    double ox = a[0] / s1, oy = a[1] / s1;
    if (a[2] < 0.0) {
        const double tx = ox;
        ox = (1.0 - std::fabs(oy)) * (tx >= 0.0 ? 1.0 : -1.0);
        oy = (1.0 - std::fabs(tx)) * (oy >= 0.0 ? 1.0 : -1.0);
    }
    const uint32_t qx = static_cast<uint32_t>(std::lround((ox + 1.0) * 0.5 * 511.0));
    const uint32_t qy = static_cast<uint32_t>(std::lround((oy + 1.0) * 0.5 * 511.0));
    const v3 dec = coneAxis(qx | (qy << 9));
    const double dl = std::sqrt(double(dec.x) * dec.x + double(dec.y) * dec.y + double(dec.z) * dec.z);
    const double ax[3] = {dec.x / dl, dec.y / dl, dec.z / dl};
    double cosMin = 1.0;
    for (const auto& u : ns) cosMin = std::min(cosMin, std::fabs(u[0] * ax[0] + u[1] * ax[1] + u[2] * ax[2]));
    // psi = acos(cosMin) widened by 2e-3 rad (the kernel's float evaluation of the bound)
    const double psi = std::acos(std::min(1.0, cosMin)) + 2e-3;
    const double qCode = psi >= 1.5707963267948966 ? 127.0 : std::ceil(std::sin(psi) * 126.0 + 1e-9);
    if (qCode > 126.0) return kConeNever;
    return qx | (qy << 9) | (static_cast<uint32_t>(qCode) << 18) | (static_cast<uint32_t>(kCode) << 25);
}
}  // namespace

void cullRecord(const std::vector<HTriangle>& tris, const std::vector<std::array<int32_t, 2>>& ranges,
                const double ctr[3], double hd, float out[6]) {
    const float never[6] = {0.0F, 0.0F, 0.0F, 1.0F, 0.0F, 0.0F};
    std::copy(never, never + 6, out);
    double kMax = 1.0;
    double m[3][3] = {};  // sum of n n^T over unit normals (lines: sign-free)
    std::vector<std::array<double, 3>> ns;
    for (const auto& rg : ranges) {
        for (int32_t i = rg[0]; i < rg[1]; ++i) {
            const HTriangle& t = tris[static_cast<size_t>(i)];
            const double ab[3] = {t.AB.x, t.AB.y, t.AB.z}, ac[3] = {t.AC.x, t.AC.y, t.AC.z};
            const double n[3] = {ab[1] * ac[2] - ab[2] * ac[1], ab[2] * ac[0] - ab[0] * ac[2],
                                 ab[0] * ac[1] - ab[1] * ac[0]};
            const double len = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            const double l1 = (std::fabs(ab[0]) + std::fabs(ab[1]) + std::fabs(ab[2])) *
                              (std::fabs(ac[0]) + std::fabs(ac[1]) + std::fabs(ac[2]));
            if (!(len > 0.0) || !std::isfinite(l1)) return;
            kMax = std::max(kMax, l1 / len);
            const std::array<double, 3> u{n[0] / len, n[1] / len, n[2] / len};
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) m[r][c] += u[static_cast<size_t>(r)] * u[static_cast<size_t>(c)];
            ns.push_back(u);
        }
    }
    if (ns.empty()) return;
    int col = 0;
    for (int c = 1; c < 3; ++c)
        if (m[c][c] > m[col][col]) col = c;
    double a[3] = {m[0][col], m[1][col], m[2][col]};
    for (int it = 0; it < 64; ++it) {
        double b[3];
        for (int r = 0; r < 3; ++r) b[r] = m[r][0] * a[0] + m[r][1] * a[1] + m[r][2] * a[2];
        const double l = std::sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
        if (!(l > 0.0)) return;
        for (int r = 0; r < 3; ++r) a[r] = b[r] / l;
    }
    double cosMin = 1.0;
    for (const auto& u : ns) cosMin = std::min(cosMin, std::fabs(u[0] * a[0] + u[1] * a[1] + u[2] * a[2]));
    // psi widened by 1e-3 rad: the float storage of a' and q, and the kernel's float evaluation
    const double psi = std::acos(std::min(1.0, cosMin)) + 1e-3;
    if (psi >= 1.5) return;
    const double cq = std::cos(psi), q = std::sin(psi);
    const double D = 2.0 * hd * 1.0002 + 0x1p-20 * (std::fabs(ctr[0]) + std::fabs(ctr[1]) + std::fabs(ctr[2]) + hd);
    const double Kc = 0x1p-18 * kMax * 1.001;
    auto up = [](double x) { return std::nextafter(static_cast<float>(x), std::numeric_limits<float>::infinity()); };
    if (!std::isfinite(D) || !std::isfinite(Kc)) return;
    out[0] = static_cast<float>(a[0] * cq);
    out[1] = static_cast<float>(a[1] * cq);
    out[2] = static_cast<float>(a[2] * cq);
    out[3] = up(q);
    out[4] = up(Kc);
    out[5] = up(D);
}

void leafCullRecord(const std::vector<HTriangle>& tris, size_t lo, size_t hi, const HAABB& box, float out[6]) {
    const double ctr[3] = {0.5 * (double(box.mn.x) + box.mx.x), 0.5 * (double(box.mn.y) + box.mx.y),
                           0.5 * (double(box.mn.z) + box.mx.z)};
    const double dx = double(box.mx.x) - box.mn.x, dy = double(box.mx.y) - box.mn.y, dz = double(box.mx.z) - box.mn.z;
    const double hd = 0.5 * std::sqrt(dx * dx + dy * dy + dz * dz);
    cullRecord(tris, {{static_cast<int32_t>(lo), static_cast<int32_t>(hi)}}, ctr, hd, out);
}

// A second topology over the reference tree's leaves ("walk tree").
// Reachability of a triangle in the reference walk is its leaf box passing the slab test: every
// ancestor box contains the leaf box coordinatewise, and for a ray with finite 1/d each computed
// slab interval grows monotonically with the box (correctly rounded - and * are monotone), so an
// ancestor passes whenever the leaf does (BVH.hpp:327-384 tests the root, then child boxes).  Any
// tree whose leaves are the reference leaves (same primitive ranges, same boxes) and whose inner
// boxes are exact unions of the leaf boxes below therefore reaches exactly the reference's
// triangles for such rays.  This one is grouped by a full-sweep SAH over the leaf centroids
// (the reference groups triangles with 10 centroid buckets, BVH.hpp:197-240).
std::vector<HBVHNode> rebuildOverLeaves(const std::vector<HBVHNode>& ref, int weight) {
    if (ref.size() <= 1) return ref;
    struct Leaf {
        HAABB box;
        v3 c;
        int32_t first, count;
    };
    std::vector<Leaf> leaves;
    for (const HBVHNode& n : ref) {
        if (n.numPrimitives > 0) {
            const v3 c{0.5F * (n.box.mn.x + n.box.mx.x), 0.5F * (n.box.mn.y + n.box.mx.y), 0.5F * (n.box.mn.z + n.box.mx.z)};
            leaves.push_back(Leaf{n.box, c, n.indexOffset, n.numPrimitives});
        }
    }
    const size_t n = leaves.size();
    auto unite = [](const HAABB& a, const HAABB& b) { return HAABB{vmin(a.mn, b.mn), vmax(a.mx, b.mx)}; };
    auto area = [](const HAABB& b) {
        const double dx = static_cast<double>(b.mx.x) - b.mn.x, dy = static_cast<double>(b.mx.y) - b.mn.y,
                     dz = static_cast<double>(b.mx.z) - b.mn.z;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    };
    std::vector<int32_t> idx(n);
    for (size_t i = 0; i < n; ++i) idx[i] = static_cast<int32_t>(i);
    std::vector<HBVHNode> out(1);
    struct Task {
        int32_t node, b, e;
    };
    std::vector<Task> st{{0, 0, static_cast<int32_t>(n)}};
    std::vector<double> rightArea(n + 1);
    std::vector<int32_t> tmp(n);
    while (!st.empty()) {
        const Task t = st.back();
        st.pop_back();
        HAABB box = leaves[static_cast<size_t>(idx[static_cast<size_t>(t.b)])].box;
        for (int32_t i = t.b + 1; i < t.e; ++i) box = unite(box, leaves[static_cast<size_t>(idx[static_cast<size_t>(i)])].box);
        if (t.e - t.b == 1) {
            const Leaf& l = leaves[static_cast<size_t>(idx[static_cast<size_t>(t.b)])];
            out[static_cast<size_t>(t.node)] = HBVHNode{l.box, l.first, l.count};
            continue;
        }
        double best = 1e300;
        int bestAxis = 0;
        int32_t bestSplit = t.b + (t.e - t.b) / 2;
        for (int axis = 0; axis < 3; ++axis) {
            std::copy(idx.begin() + t.b, idx.begin() + t.e, tmp.begin() + t.b);
            std::stable_sort(tmp.begin() + t.b, tmp.begin() + t.e, [&](int32_t x, int32_t y) {
                return comp(leaves[static_cast<size_t>(x)].c, axis) < comp(leaves[static_cast<size_t>(y)].c, axis);
            });
            HAABB acc = leaves[static_cast<size_t>(tmp[static_cast<size_t>(t.e - 1)])].box;
            rightArea[static_cast<size_t>(t.e - 1)] = area(acc);
            for (int32_t i = t.e - 2; i > t.b; --i) {
                acc = unite(acc, leaves[static_cast<size_t>(tmp[static_cast<size_t>(i)])].box);
                rightArea[static_cast<size_t>(i)] = area(acc);
            }
            // weights: 0 one per leaf, 1 the leaf's triangle count, 2 one + count
            auto wt = [&](int32_t i) {
                const int32_t c = leaves[static_cast<size_t>(tmp[static_cast<size_t>(i)])].count;
                return weight == 0 ? 1.0 : (weight == 1 ? static_cast<double>(c) : 1.0 + c);
            };
            double wTotal = 0.0;
            for (int32_t i = t.b; i < t.e; ++i) wTotal += wt(i);
            double wLeft = 0.0;
            acc = leaves[static_cast<size_t>(tmp[static_cast<size_t>(t.b)])].box;
            for (int32_t i = t.b + 1; i < t.e; ++i) {  // split: [b, i) | [i, e)
                wLeft += wt(i - 1);
                const double cost = area(acc) * wLeft + rightArea[static_cast<size_t>(i)] * (wTotal - wLeft);
                if (cost < best) {
                    best = cost;
                    bestAxis = axis;
                    bestSplit = i;
                }
                acc = unite(acc, leaves[static_cast<size_t>(tmp[static_cast<size_t>(i)])].box);
            }
        }
        std::stable_sort(idx.begin() + t.b, idx.begin() + t.e, [&](int32_t x, int32_t y) {
            return comp(leaves[static_cast<size_t>(x)].c, bestAxis) < comp(leaves[static_cast<size_t>(y)].c, bestAxis);
        });
        const int32_t left = static_cast<int32_t>(out.size());
        out.resize(out.size() + 2);
        out[static_cast<size_t>(t.node)] = HBVHNode{box, left, 0};
        st.push_back({left + 1, bestSplit, t.e});
        st.push_back({left, t.b, bestSplit});
    }
    return out;
}

// Insertion-based optimisation of a BVH2 over fixed leaves (Bittner, Hapala, Havran 2013).  In the
// exact mode no inner node is culled, so a ray visits every inner node whose box it passes: for
// rays spread over the scene the expected visits are the summed inner-node surface area over the
// root's, the quantity the SAH sweep above approximates greedily and this pass lowers.  Each round
// takes a batch of inner nodes (below), removes each (its sibling takes the parent's
// place) and reinserts its two children, one at a time, as the sibling of the node where the summed
// area grows least (a branch-and-bound search from the root); boxes stay exact unions, the leaves
// are untouched.  Rounds stop after three in a row that lower the total by less than 0.001 %.
#ifndef MRT_TREE_OPT_STOP
#define MRT_TREE_OPT_STOP 0.99999
#endif
constexpr double kTreeOptStop = MRT_TREE_OPT_STOP;  // a round must lower the summed area below this fraction
#ifndef MRT_TREE_OPT_BATCH
#define MRT_TREE_OPT_BATCH 100
#endif
constexpr size_t kTreeOptBatchDiv = MRT_TREE_OPT_BATCH;  // a round moves 1 / this of the candidates
std::vector<HBVHNode> optimizeOverLeaves(const std::vector<HBVHNode>& in, int rounds, bool bounded) {
    if (in.size() < 8 || rounds <= 0) return in;
    struct N {
        HAABB box;
        int32_t l = -1, r = -1, parent = -1;
        int32_t first = 0, count = 0;  // leaf: primitive range
        int32_t height = 0;            // longest path to a leaf below (leaves 0)
    };
    // the nodes reachable from the root (a build's array may hold unused zero slots), renumbered
    // parents first
    std::vector<N> t;
    {
        std::vector<std::pair<int32_t, int32_t>> st{{0, -1}};  // (input node, parent in t)
        while (!st.empty()) {
            const auto [i, parent] = st.back();
            st.pop_back();
            const int32_t k = static_cast<int32_t>(t.size());
            t.emplace_back();
            N& n = t.back();
            const HBVHNode& h = in[static_cast<size_t>(i)];
            n.box = h.box;
            n.parent = parent;
            if (parent >= 0) {
                N& pn = t[static_cast<size_t>(parent)];
                (pn.l < 0 ? pn.l : pn.r) = k;
            }
            if (h.numPrimitives > 0) {
                n.first = h.indexOffset;
                n.count = h.numPrimitives;
            } else {
                st.push_back({h.indexOffset + 1, k});
                st.push_back({h.indexOffset, k});
            }
        }
    }
    auto unite = [](const HAABB& a, const HAABB& b) { return HAABB{vmin(a.mn, b.mn), vmax(a.mx, b.mx)}; };
    auto area = [](const HAABB& b) {
        const double dx = static_cast<double>(b.mx.x) - b.mn.x, dy = static_cast<double>(b.mx.y) - b.mn.y,
                     dz = static_cast<double>(b.mx.z) - b.mn.z;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    };
    int32_t root = 0;
    auto refit = [&](int32_t i) {
        for (; i >= 0; i = t[static_cast<size_t>(i)].parent) {
            N& n = t[static_cast<size_t>(i)];
            n.box = unite(t[static_cast<size_t>(n.l)].box, t[static_cast<size_t>(n.r)].box);
            n.height = 1 + std::max(t[static_cast<size_t>(n.l)].height, t[static_cast<size_t>(n.r)].height);
        }
    };
    {  // heights bottom-up (children have larger indices: parents first above)
        for (size_t k = t.size(); k-- > 0;) {
            N& n = t[k];
            if (n.count == 0 && n.l >= 0)
                n.height = 1 + std::max(t[static_cast<size_t>(n.l)].height, t[static_cast<size_t>(n.r)].height);
        }
    }
    // The walk's traversal stack grows with the tree's depth (3 pushes per wide level at most; entries
    // past the LDS part spill to global memory, and the packet walk's stack is bounded), so a
    // bounded optimisation searches only positions that keep the tree within the sweep's height (the
    // fallbacks below usually do too; walkTreeBuild rejects any result whose wide tree is deeper).
    const int32_t maxHeight = bounded ? t[0].height : std::numeric_limits<int32_t>::max() / 4;
    auto total = [&]() {
        double a = 0.0;
        for (const N& n : t)
            if (n.count == 0 && n.l >= 0) a += area(n.box);
        return a;
    };
    // the best sibling for subtree x: minimal area of the new parent plus the growth of every ancestor
    // within the height bound (fallback, when the bounded search finds none: a position that keeps
    // the height, chosen by the caller below)
    auto bestSibling = [&](int32_t x, int32_t fallback) {
        const HAABB bx = t[static_cast<size_t>(x)].box;
        const double ax = area(bx);
        const int32_t hx = t[static_cast<size_t>(x)].height;
        struct Q {
            double bound, induced;
            int32_t node, depth;
            bool operator<(const Q& o) const { return bound > o.bound; }
        };
        std::priority_queue<Q> pq;
        pq.push(Q{ax, 0.0, root, 0});
        double best = std::numeric_limits<double>::infinity();
        int32_t bestNode = -1;
        while (!pq.empty()) {
            const Q q = pq.top();
            pq.pop();
            if (q.bound >= best) break;
            const N& c = t[static_cast<size_t>(q.node)];
            const double merged = area(unite(c.box, bx));
            const double cost = q.induced + merged;
            // the new parent sits at c's depth: x and c's subtree one level down
            if (cost < best && q.depth + 1 + std::max(hx, c.height) <= maxHeight) {
                best = cost;
                bestNode = q.node;
            }
            if (c.count == 0 && c.l >= 0 && q.depth + 2 + hx <= maxHeight) {
                const double ind = q.induced + merged - area(c.box);
                const double bound = ind + ax;
                if (bound < best) {
                    pq.push(Q{bound, ind, c.l, q.depth + 1});
                    pq.push(Q{bound, ind, c.r, q.depth + 1});
                }
            }
        }
        return bestNode >= 0 ? bestNode : fallback;
    };
    // x becomes the sibling of c under the (free) node p
    auto insertAt = [&](int32_t x, int32_t c, int32_t p) {
        const int32_t g = t[static_cast<size_t>(c)].parent;
        N& np = t[static_cast<size_t>(p)];
        np.l = c;
        np.r = x;
        np.count = 0;
        np.parent = g;
        np.height = 1 + std::max(t[static_cast<size_t>(c)].height, t[static_cast<size_t>(x)].height);
        t[static_cast<size_t>(c)].parent = p;
        t[static_cast<size_t>(x)].parent = p;
        if (g < 0) {
            root = p;
        } else if (t[static_cast<size_t>(g)].l == c) {
            t[static_cast<size_t>(g)].l = p;
        } else {
            t[static_cast<size_t>(g)].r = p;
        }
        refit(p);
    };
    double cur = total();
    std::vector<int> stamp(t.size(), -100);  // the round a node was last taken out
    int stale = 0;
    for (int round = 0; round < rounds; ++round) {
        // the batch: the 1 % of inner nodes below the root's children that fit their children worst
        // (Bittner et al.'s m_min * m_sum * m_area: large, and much larger than its children), skipping
        // the nodes moved in the last two rounds
        std::vector<std::pair<double, int32_t>> cand;
        for (size_t i = 0; i < t.size(); ++i) {
            const N& n = t[i];
            if (n.count != 0 || n.l < 0 || static_cast<int32_t>(i) == root || n.parent < 0 || n.parent == root) continue;
            if (stamp[i] >= round - 2) continue;
            const double a = area(n.box), al = area(t[static_cast<size_t>(n.l)].box), ar = area(t[static_cast<size_t>(n.r)].box);
            const double m = (a / std::max(1e-30, std::min(al, ar))) * (a / std::max(1e-30, al + ar)) * a;
            cand.push_back({m, static_cast<int32_t>(i)});
        }
        const size_t batch = std::max<size_t>(1, cand.size() / kTreeOptBatchDiv);
        std::partial_sort(cand.begin(), cand.begin() + static_cast<std::ptrdiff_t>(std::min(batch, cand.size())), cand.end(),
                          [](const auto& a, const auto& b) { return a.first > b.first; });
        for (size_t k = 0; k < batch && k < cand.size(); ++k) {
            const int32_t v = cand[k].second;
            stamp[static_cast<size_t>(v)] = round;
            N& nv = t[static_cast<size_t>(v)];
            if (nv.count != 0 || nv.l < 0 || v == root || nv.parent < 0 || nv.parent == root) continue;
            // remove v and its parent p: v's sibling takes p's place; v and p become free parents
            const int32_t p = nv.parent;
            const int32_t sib = t[static_cast<size_t>(p)].l == v ? t[static_cast<size_t>(p)].r : t[static_cast<size_t>(p)].l;
            const int32_t g = t[static_cast<size_t>(p)].parent;
            if (t[static_cast<size_t>(g)].l == p) t[static_cast<size_t>(g)].l = sib; else t[static_cast<size_t>(g)].r = sib;
            t[static_cast<size_t>(sib)].parent = g;
            refit(g);
            const int32_t a = nv.l, b = nv.r;
            // reinsert the larger child first
            const bool aFirst = area(t[static_cast<size_t>(a)].box) >= area(t[static_cast<size_t>(b)].box);
            const int32_t x1 = aFirst ? a : b, x2 = aFirst ? b : a;
            t[static_cast<size_t>(x1)].parent = -1;
            t[static_cast<size_t>(x2)].parent = -1;
            nv.l = nv.r = -1;
            // Fallbacks that keep every height at most what it was before v was taken out: sib now
            // stands where p stood, so x1 beside sib sits one level higher than under v.  If x1 went
            // there, x2 beside x1 rebuilds the old shape (sib beside the pair x1, x2); if x1 went
            // elsewhere, x2 beside sib is one level higher than under v - unless x1 went into sib's
            // subtree, whose new height the search checked at sib's depth, not one below.  So the
            // fallbacks usually keep the bound; the guarantee is walkTreeBuild's check of the wide
            // tree's depth, which rejects an optimised tree deeper than the sweep's.
            insertAt(x1, bestSibling(x1, sib), v);
            const bool pairAtP = t[static_cast<size_t>(v)].l == sib && t[static_cast<size_t>(v)].r == x1;
            insertAt(x2, bestSibling(x2, pairAtP ? x1 : sib), p);
        }
        const double next = total();
        stale = next > cur * kTreeOptStop ? stale + 1 : 0;
        cur = next;
        if (stale >= 3) break;
    }
    // re-emit in the reference numbering: root 0, an inner node's children adjacent
    std::vector<HBVHNode> out(1);
    std::vector<std::pair<int32_t, int32_t>> st{{root, 0}};
    while (!st.empty()) {
        const auto [i, slot] = st.back();
        st.pop_back();
        const N& n = t[static_cast<size_t>(i)];
        if (n.count > 0) {
            out[static_cast<size_t>(slot)] = HBVHNode{n.box, n.first, n.count};
            continue;
        }
        const int32_t left = static_cast<int32_t>(out.size());
        out.resize(out.size() + 2);
        out[static_cast<size_t>(slot)] = HBVHNode{n.box, left, 0};
        st.push_back({n.r, left + 1});
        st.push_back({n.l, left});
    }
    return out;
}

// Rotations of a BVH2 over fixed leaves that lower the optimal 4-wide collapse's summed area
// directly (the insertion pass above lowers the BVH2's): at each inner node n the four rotations
// that swap one child with a grandchild under the other (Kopta et al. 2012), kept when the root's
// collapse cost falls.  The collapse's forest table (collapseForests) of a node depends on its
// subtree only, so a rotation recomputes the rotated child, n and n's ancestors.
static std::vector<HBVHNode> rotateForWide(const std::vector<HBVHNode>& in, int sweeps) {
    if (in.size() < 8 || sweeps <= 0) return in;
    constexpr int W1 = kWalkWidth + 1;
    struct R {
        HAABB box;
        int32_t l = -1, r = -1, parent = -1, first = 0, count = 0;
        double F[W1] = {};
    };
    std::vector<R> t;
    {
        std::vector<std::pair<int32_t, int32_t>> st{{0, -1}};
        while (!st.empty()) {
            const auto [i, parent] = st.back();
            st.pop_back();
            const int32_t k = static_cast<int32_t>(t.size());
            t.emplace_back();
            R& n = t.back();
            const HBVHNode& h = in[static_cast<size_t>(i)];
            n.box = h.box;
            n.parent = parent;
            if (parent >= 0) {
                R& pn = t[static_cast<size_t>(parent)];
                (pn.l < 0 ? pn.l : pn.r) = k;
            }
            if (h.numPrimitives > 0) {
                n.first = h.indexOffset;
                n.count = h.numPrimitives;
            } else {
                st.push_back({h.indexOffset + 1, k});
                st.push_back({h.indexOffset, k});
            }
        }
    }
    auto area = [](const HAABB& b) {
        const double dx = static_cast<double>(b.mx.x) - b.mn.x, dy = static_cast<double>(b.mx.y) - b.mn.y,
                     dz = static_cast<double>(b.mx.z) - b.mn.z;
        return dx * dy + dy * dz + dz * dx;
    };
    auto inner = [&](int32_t i) { return t[static_cast<size_t>(i)].count == 0; };
    auto dp = [&](int32_t i) {  // collapseForests' recurrence for node i from its children's rows
        R& n = t[static_cast<size_t>(i)];
        if (n.count > 0) return;
        n.box = HAABB{vmin(t[static_cast<size_t>(n.l)].box.mn, t[static_cast<size_t>(n.r)].box.mn),
                      vmax(t[static_cast<size_t>(n.l)].box.mx, t[static_cast<size_t>(n.r)].box.mx)};
        const double* L = t[static_cast<size_t>(n.l)].F;
        const double* Rr = t[static_cast<size_t>(n.r)].F;
        auto best = [&](int j) {
            double c = std::numeric_limits<double>::infinity();
            for (int a = 1; a < j; ++a) c = std::min(c, L[a] + Rr[j - a]);
            return c;
        };
        const double asWide = area(n.box) + best(kWalkWidth);
        n.F[1] = asWide;
        for (int j = 2; j < W1; ++j) n.F[j] = std::min(asWide, best(j));
    };
    for (size_t k = t.size(); k-- > 0;) dp(static_cast<int32_t>(k));  // children after parents
    auto up = [&](int32_t i) {
        for (; i >= 0; i = t[static_cast<size_t>(i)].parent) dp(i);
    };
    // swap subtree x (child of n) with y (child of n's other child m)
    auto swapSub = [&](int32_t n, int32_t x, int32_t m, int32_t y) {
        R& rn = t[static_cast<size_t>(n)];
        R& rm = t[static_cast<size_t>(m)];
        (rn.l == x ? rn.l : rn.r) = y;
        (rm.l == y ? rm.l : rm.r) = x;
        t[static_cast<size_t>(x)].parent = m;
        t[static_cast<size_t>(y)].parent = n;
        dp(m);
        up(n);
    };
    double cur = t[0].F[1];
    for (int sweep = 0; sweep < sweeps; ++sweep) {
        int improved = 0;
        for (int32_t n = 0; n < static_cast<int32_t>(t.size()); ++n) {
            if (!inner(n)) continue;
            for (int side = 0; side < 2; ++side) {
                const int32_t x = side == 0 ? t[static_cast<size_t>(n)].l : t[static_cast<size_t>(n)].r;
                const int32_t m = side == 0 ? t[static_cast<size_t>(n)].r : t[static_cast<size_t>(n)].l;
                if (!inner(m)) continue;
                bool done = false;
                for (int g = 0; g < 2 && !done; ++g) {
                    const int32_t y = g == 0 ? t[static_cast<size_t>(m)].l : t[static_cast<size_t>(m)].r;
                    swapSub(n, x, m, y);
                    if (t[0].F[1] < cur * (1.0 - 1e-12)) {
                        cur = t[0].F[1];
                        ++improved;
                        done = true;
                    } else {
                        swapSub(n, y, m, x);  // undo
                    }
                }
                if (done) break;
            }
        }
        if (improved == 0) break;
    }
    std::vector<HBVHNode> out(1);
    std::vector<std::pair<int32_t, int32_t>> st{{0, 0}};
    while (!st.empty()) {
        const auto [i, slot] = st.back();
        st.pop_back();
        const R& n = t[static_cast<size_t>(i)];
        if (n.count > 0) {
            out[static_cast<size_t>(slot)] = HBVHNode{n.box, n.first, n.count};
            continue;
        }
        const int32_t left = static_cast<int32_t>(out.size());
        out.resize(out.size() + 2);
        out[static_cast<size_t>(slot)] = HBVHNode{n.box, left, 0};
        st.push_back({n.r, left + 1});
        st.push_back({n.l, left});
    }
    return out;
}

namespace {
// the slab entry of a box (t >= 0), or +inf when the half-line misses it
float halfLineEntry(const HAABB& b, v3 o, v3 inv) {
    float t0 = 0.0F, t1 = std::numeric_limits<float>::infinity();
    for (int a = 0; a < 3; ++a) {
        const float lo = (comp(b.mn, a) - comp(o, a)) * comp(inv, a), hi = (comp(b.mx, a) - comp(o, a)) * comp(inv, a);
        t0 = std::max(t0, std::min(lo, hi));
        t1 = std::min(t1, std::max(lo, hi));
    }
    return t0 <= t1 ? t0 : std::numeric_limits<float>::infinity();
}
}  // namespace

std::vector<SampleRay> sampleFrameRays(const std::vector<HBVHNode>& nodes, const HScene& sc, const GCamera& cam,
                                       int maxDepth) {
    using Ray = SampleRay;
    std::vector<Ray> rays;
    if (nodes.empty() || sc.triangles.empty()) return rays;
    auto inner = [&](size_t i) { return nodes[i].numPrimitives == 0 && nodes.size() > 1; };
    const auto entry = halfLineEntry;
    auto triHit = [](const HTriangle& t, v3 o, v3 d, float* tOut) {  // Moller-Trumbore, float
        const v3 p = cross(d, t.AC);
        const float det = dot(t.AB, p);
        if (std::fabs(det) < 1e-9F) return false;
        const float inv = 1.0F / det;
        const v3 s = o - t.A;
        const float u = inv * dot(s, p);
        if (u < 0.0F || u > 1.0F) return false;
        const v3 q = cross(s, t.AB);
        const float v = inv * dot(d, q);
        if (v < 0.0F || u + v > 1.0F) return false;
        *tOut = inv * dot(t.AC, q);
        return *tOut > 1e-4F;
    };
    // closest hit: triangle index (BVH order), or -2 for a light, -1 for none
    auto closest = [&](v3 o, v3 d, float* tBest) {
        const v3 inv{1.0F / d.x, 1.0F / d.y, 1.0F / d.z};
        int best = -1;
        float bt = std::numeric_limits<float>::infinity();
        std::vector<int32_t> st{0};
        while (!st.empty()) {
            const size_t i = static_cast<size_t>(st.back());
            st.pop_back();
            if (!(entry(nodes[i].box, o, inv) < bt)) continue;
            if (inner(i)) {
                st.push_back(nodes[i].indexOffset + 1);
                st.push_back(nodes[i].indexOffset);
                continue;
            }
            for (int32_t k = 0; k < nodes[i].numPrimitives; ++k) {
                float t;
                const int32_t j = nodes[i].indexOffset + k;
                if (triHit(sc.triangles[static_cast<size_t>(j)], o, d, &t) && t < bt) {
                    bt = t;
                    best = j;
                }
            }
        }
        for (const HLight& l : sc.lights) {
            float t;
            if (l.kind == kAreaLight && triHit(l.tri, o, d, &t) && t < bt) {
                bt = t;
                best = -2;
            }
        }
        *tBest = bt;
        return best;
    };
    std::vector<const HLight*> areaLights;
    for (const HLight& l : sc.lights)
        if (l.kind == kAreaLight) areaLights.push_back(&l);
    // the sample: the frame's walked rays (camera rays of a 192 x 108 pixel grid, each path's
    // bounces and shadow rays); camera rays weigh 0.6 (the packet walk's cost per ray against the
    // per-lane walks', profiles/r06_bench.json), the others 1
    std::mt19937 rng(0x4D525406u);
    std::uniform_real_distribution<float> U(0.0F, 1.0F);
    // (camera weight 0.25 / 1, shadow weight 0.5 / 2, grids of 96 x 54 and 384 x 216 pixels and an
    // area floor of 0.1 % / 10 % measured within 0.5 % of these: profiles/r06_ray_collapse_ab.txt)
    constexpr float camW = 0.6F, shadowW = 1.0F;
    constexpr int gx = 192, gy = 108;
    struct Path {
        v3 o, d;
        int depth;
    };
    for (int py = 0; py < gy; ++py)
        for (int px = 0; px < gx; ++px) {
            const float u = (static_cast<float>(px) + U(rng)) / static_cast<float>(gx);
            const float v = (static_cast<float>(py) + U(rng)) / static_cast<float>(gy);
            v3 o, d;
            if (cam.kind == 1) {
                o = (cam.position + cam.right * ((u - 0.5F) * cam.hFov)) + cam.up * ((0.5F - v) * cam.vFov);
                d = cam.direction;
            } else {
                const v3 dest = ((cam.position + cam.direction) + cam.right * fastArcTan(cam.hFov * (u - 0.5F))) +
                                cam.up * fastArcTan(cam.vFov * (0.5F - v));
                o = cam.position;
                d = normalize(dest - cam.position);
            }
            std::vector<Path> work{{o, d, 1}};
            while (!work.empty()) {
                const Path p = work.back();
                work.pop_back();
                rays.push_back(Ray{p.o, p.d, p.depth == 1 ? camW : 1.0F});
                float t;
                const int hit = closest(p.o, p.d, &t);
                if (hit < 0) continue;  // a miss, or a light (emissive: no children)
                const HTriangle& tri = sc.triangles[static_cast<size_t>(hit)];
                const HMaterial m = tri.mat >= 0 && tri.mat < static_cast<int32_t>(sc.materials.size())
                                        ? sc.materials[static_cast<size_t>(tri.mat)] : HMaterial{};
                if (m.Le.x > 0.0F || m.Le.y > 0.0F || m.Le.z > 0.0F) continue;
                v3 n = normalize(cross(tri.AB, tri.AC));
                if (dot(n, p.d) > 0.0F) n = -n;
                const v3 P = p.o + p.d * t + n * 1e-3F;
                const bool diffuse = m.Kd.x > 0.0F || m.Kd.y > 0.0F || m.Kd.z > 0.0F;
                if (diffuse && !areaLights.empty()) {  // a shadow ray to a random point of a random light
                    const HLight& l = *areaLights[static_cast<size_t>(U(rng) * 0.99999F * static_cast<float>(areaLights.size()))];
                    float r1 = U(rng), r2 = U(rng);
                    if (r1 + r2 >= 1.0F) {
                        r1 = 1.0F - r1;
                        r2 = 1.0F - r2;
                    }
                    const v3 q = (l.tri.A + l.tri.AB * r1) + l.tri.AC * r2;
                    rays.push_back(Ray{P, normalize(q - P), shadowW});
                }
                if (p.depth >= maxDepth) continue;  // the depth-capped level is not walked
                if (diffuse && (p.depth <= 1 || U(rng) > 0.5F)) {  // cosine bounce (PathTracer.cpp:89-91)
                    const float phi = 6.2831853F * U(rng), r2 = U(rng);
                    const v3 a = std::fabs(n.x) > 0.1F ? v3{0.0F, 1.0F, 0.0F} : v3{1.0F, 0.0F, 0.0F};
                    const v3 tu = normalize(cross(a, n)), tv = cross(n, tu);
                    const float ct = std::sqrt(r2);
                    work.push_back(Path{P, normalize((tu * (std::cos(phi) * ct) + tv * (std::sin(phi) * ct)) + n * std::sqrt(1.0F - r2)),
                                        p.depth + 1});
                }
                if (m.Ks.x > 0.0F || m.Ks.y > 0.0F || m.Ks.z > 0.0F) work.push_back(Path{P, reflect(p.d, n), p.depth + 1});
            }
        }
    return rays;
}

std::vector<double> frameRayNodeCosts(const std::vector<HBVHNode>& nodes, const HScene& sc, const GCamera& cam,
                                      int width, int height, int maxDepth) {
    if (nodes.empty() || sc.triangles.empty() || width <= 0 || height <= 0) return std::vector<double>(nodes.size(), 0.0);
    return sampleRayNodeCosts(nodes, sampleFrameRays(nodes, sc, cam, maxDepth));
}

// the share of the root's area every node's cost carries besides its sample rays (so that nodes no
// sample ray reaches are still ordered)
constexpr float kRayCostFloor = 0.01F;

std::vector<double> sampleRayNodeCosts(const std::vector<HBVHNode>& nodes, const std::vector<SampleRay>& rays) {
    std::vector<double> cost(nodes.size(), 0.0);
    if (nodes.empty() || rays.empty()) return cost;
    auto inner = [&](size_t i) { return nodes[i].numPrimitives == 0 && nodes.size() > 1; };
    constexpr float floorW = kRayCostFloor;
    // every node whose box each sample ray's half-line passes (the exact walk culls no inner node)
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::vector<double>> part(hw, std::vector<double>(nodes.size(), 0.0));
    std::vector<std::thread> pool;
    for (unsigned w = 0; w < hw; ++w)
        pool.emplace_back([&, w] {
            std::vector<int32_t> st;
            std::vector<double>& c = part[w];
            for (size_t k = w; k < rays.size(); k += hw) {
                const SampleRay& r = rays[k];
                const v3 inv{1.0F / r.d.x, 1.0F / r.d.y, 1.0F / r.d.z};
                st.assign(1, 0);
                while (!st.empty()) {
                    const size_t i = static_cast<size_t>(st.back());
                    st.pop_back();
                    if (!(halfLineEntry(nodes[i].box, r.o, inv) < std::numeric_limits<float>::infinity())) continue;
                    c[i] += r.w;
                    if (inner(i)) {
                        st.push_back(nodes[i].indexOffset);
                        st.push_back(nodes[i].indexOffset + 1);
                    }
                }
            }
        });
    for (std::thread& t : pool) t.join();
    double total = 0.0;
    for (const SampleRay& r : rays) total += r.w;
    auto area = [&](size_t i) {
        const HAABB& b = nodes[i].box;
        const double dx = static_cast<double>(b.mx.x) - b.mn.x, dy = static_cast<double>(b.mx.y) - b.mn.y,
                     dz = static_cast<double>(b.mx.z) - b.mn.z;
        return dx * dy + dy * dz + dz * dx;
    };
    const double rootArea = std::max(1e-30, area(0));
    for (size_t i = 0; i < nodes.size(); ++i) {
        double s = 0.0;
        for (unsigned w = 0; w < hw; ++w) s += part[w][i];
        cost[i] = s + floorW * total * area(i) / rootArea;
    }
    return cost;
}

// Rotations of the walk tree's BVH2 (Kopta et al.'s four per inner node, as rotateForWide) kept where
// they lower the optimal 4-wide collapse's cost under the frame's ray sample: a node costs the summed
// weight of the sample half-lines that pass its box, plus kRayCostFloor of its share of the root's
// area (sampleRayNodeCosts' cost, the one toQuantizedBVH4 collapses with).  A rotation at n changes
// one box, that of n's child m, and every ray passing m's new box passes n's: m's rays are re-counted
// from n's list.  Leaves and their boxes are untouched and inner boxes stay exact unions (the walk
// tree's exactness argument); no rotation makes a subtree taller than it was.
std::vector<HBVHNode> rotateForRays(const std::vector<HBVHNode>& in, const std::vector<SampleRay>& rays, int sweeps) {
    if (in.size() < 8 || sweeps <= 0 || rays.empty() || in[0].numPrimitives > 0) return in;
    constexpr int W1 = kWalkWidth + 1;
    struct R {
        HAABB box;
        int32_t l = -1, r = -1, parent = -1, first = 0, count = 0;
        int32_t height = 0, maxHeight = 0;  // maxHeight: the input's height of this node (a bound)
        double cost = 0.0;
        double F[W1] = {};
    };
    std::vector<R> t;
    {
        std::vector<std::pair<int32_t, int32_t>> st{{0, -1}};
        while (!st.empty()) {
            const auto [i, parent] = st.back();
            st.pop_back();
            const int32_t k = static_cast<int32_t>(t.size());
            t.emplace_back();
            R& n = t.back();
            const HBVHNode& h = in[static_cast<size_t>(i)];
            n.box = h.box;
            n.parent = parent;
            if (parent >= 0) {
                R& pn = t[static_cast<size_t>(parent)];
                (pn.l < 0 ? pn.l : pn.r) = k;
            }
            if (h.numPrimitives > 0) {
                n.first = h.indexOffset;
                n.count = h.numPrimitives;
            } else {
                st.push_back({h.indexOffset + 1, k});
                st.push_back({h.indexOffset, k});
            }
        }
    }
    const size_t nn = t.size();
    auto inner = [&](int32_t i) { return t[static_cast<size_t>(i)].count == 0; };
    for (size_t k = nn; k-- > 0;) {  // heights, children after parents
        R& n = t[k];
        if (n.count == 0)
            n.height = 1 + std::max(t[static_cast<size_t>(n.l)].height, t[static_cast<size_t>(n.r)].height);
        n.maxHeight = n.height;
    }
    auto area = [](const HAABB& b) {
        const double dx = static_cast<double>(b.mx.x) - b.mn.x, dy = static_cast<double>(b.mx.y) - b.mn.y,
                     dz = static_cast<double>(b.mx.z) - b.mn.z;
        return dx * dy + dy * dz + dz * dx;
    };
    double total = 0.0;
    for (const SampleRay& ry : rays) total += ry.w;
    const double rootArea = std::max(1e-30, area(t[0].box));
    const double floorK = kRayCostFloor * total / rootArea;
    std::vector<v3> inv(rays.size());
    for (size_t k = 0; k < rays.size(); ++k) inv[k] = v3{1.0F / rays[k].d.x, 1.0F / rays[k].d.y, 1.0F / rays[k].d.z};
    auto passes = [&](const HAABB& b, int32_t k) {
        return halfLineEntry(b, rays[static_cast<size_t>(k)].o, inv[static_cast<size_t>(k)]) < std::numeric_limits<float>::infinity();
    };
    // every inner node's sample rays (ids), by one walk per ray over the tree (threads over rays)
    std::vector<std::vector<int32_t>> list(nn);
    {
        const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::vector<std::vector<int32_t>>> part(hw);
        std::vector<std::thread> pool;
        for (unsigned w = 0; w < hw; ++w)
            pool.emplace_back([&, w] {
                std::vector<std::vector<int32_t>>& pl = part[w];
                pl.assign(nn, {});
                std::vector<int32_t> st;
                for (size_t k = w; k < rays.size(); k += hw) {
                    st.assign(1, 0);
                    while (!st.empty()) {
                        const int32_t i = st.back();
                        st.pop_back();
                        const R& n = t[static_cast<size_t>(i)];
                        if (n.count > 0 || !passes(n.box, static_cast<int32_t>(k))) continue;
                        pl[static_cast<size_t>(i)].push_back(static_cast<int32_t>(k));
                        st.push_back(n.l);
                        st.push_back(n.r);
                    }
                }
            });
        for (std::thread& th : pool) th.join();
        for (size_t i = 0; i < nn; ++i) {
            size_t sz = 0;
            for (unsigned w = 0; w < hw; ++w) sz += part[w][i].size();
            list[i].reserve(sz);
            for (unsigned w = 0; w < hw; ++w) list[i].insert(list[i].end(), part[w][i].begin(), part[w][i].end());
            std::sort(list[i].begin(), list[i].end());
        }
    }
    auto weigh = [&](const std::vector<int32_t>& ids, const HAABB& b) {
        double c = 0.0;
        for (const int32_t k : ids) c += rays[static_cast<size_t>(k)].w;
        return c + floorK * area(b);
    };
    for (size_t i = 0; i < nn; ++i)
        if (t[i].count == 0) t[i].cost = weigh(list[i], t[i].box);
    auto dp = [&](int32_t i) {  // collapseForests' recurrence, node costs instead of areas
        R& n = t[static_cast<size_t>(i)];
        if (n.count > 0) return;
        const R& a = t[static_cast<size_t>(n.l)];
        const R& b = t[static_cast<size_t>(n.r)];
        n.height = 1 + std::max(a.height, b.height);
        auto best = [&](int j) {
            double c = std::numeric_limits<double>::infinity();
            for (int q = 1; q < j; ++q) c = std::min(c, a.F[q] + b.F[j - q]);
            return c;
        };
        const double asWide = n.cost + best(kWalkWidth);
        n.F[1] = asWide;
        for (int j = 2; j < W1; ++j) n.F[j] = std::min(asWide, best(j));
    };
    for (size_t k = nn; k-- > 0;) dp(static_cast<int32_t>(k));
    auto up = [&](int32_t i) {
        for (; i >= 0; i = t[static_cast<size_t>(i)].parent) dp(i);
    };
    std::vector<int32_t> keep;
    double cur = t[0].F[1];
    for (int sweep = 0; sweep < sweeps; ++sweep) {
        int improved = 0;
        for (int32_t n = 0; n < static_cast<int32_t>(nn); ++n) {
            if (!inner(n)) continue;
            for (int side = 0; side < 2; ++side) {
                const int32_t x = side == 0 ? t[static_cast<size_t>(n)].l : t[static_cast<size_t>(n)].r;
                const int32_t m = side == 0 ? t[static_cast<size_t>(n)].r : t[static_cast<size_t>(n)].l;
                if (!inner(m)) continue;
                bool done = false;
                for (int g = 0; g < 2 && !done; ++g) {
                    const int32_t y = g == 0 ? t[static_cast<size_t>(m)].l : t[static_cast<size_t>(m)].r;
                    const int32_t z = g == 0 ? t[static_cast<size_t>(m)].r : t[static_cast<size_t>(m)].l;  // stays under m
                    // after the swap m holds x and z, n holds y and m: the heights must stay within bounds
                    const int32_t hm = 1 + std::max(t[static_cast<size_t>(x)].height, t[static_cast<size_t>(z)].height);
                    if (hm > t[static_cast<size_t>(m)].maxHeight ||
                        1 + std::max(hm, t[static_cast<size_t>(y)].height) > t[static_cast<size_t>(n)].maxHeight)
                        continue;
                    const HAABB mb{vmin(t[static_cast<size_t>(x)].box.mn, t[static_cast<size_t>(z)].box.mn),
                                   vmax(t[static_cast<size_t>(x)].box.mx, t[static_cast<size_t>(z)].box.mx)};
                    keep.clear();
                    for (const int32_t k : list[static_cast<size_t>(n)])
                        if (passes(mb, k)) keep.push_back(k);
                    const double newCost = weigh(keep, mb);
                    R& rn = t[static_cast<size_t>(n)];
                    R& rm = t[static_cast<size_t>(m)];
                    const HAABB oldBox = rm.box;
                    const double oldCost = rm.cost;
                    auto link = [&](int32_t a, int32_t b) {  // swap a (under n) with b (under m)
                        (rn.l == a ? rn.l : rn.r) = b;
                        (rm.l == b ? rm.l : rm.r) = a;
                        t[static_cast<size_t>(a)].parent = m;
                        t[static_cast<size_t>(b)].parent = n;
                    };
                    link(x, y);
                    rm.box = mb;
                    rm.cost = newCost;
                    dp(m);
                    up(n);
                    if (t[0].F[1] < cur * (1.0 - 1e-9)) {
                        cur = t[0].F[1];
                        list[static_cast<size_t>(m)].swap(keep);
                        ++improved;
                        done = true;
                    } else {  // undo
                        link(y, x);
                        rm.box = oldBox;
                        rm.cost = oldCost;
                        dp(m);
                        up(n);
                    }
                }
                if (done) break;
            }
        }
        if (improved == 0) break;
    }
    std::vector<HBVHNode> out(1);
    std::vector<std::pair<int32_t, int32_t>> st{{0, 0}};
    while (!st.empty()) {
        const auto [i, slot] = st.back();
        st.pop_back();
        const R& n = t[static_cast<size_t>(i)];
        if (n.count > 0) {
            out[static_cast<size_t>(slot)] = HBVHNode{n.box, n.first, n.count};
            continue;
        }
        const int32_t left = static_cast<int32_t>(out.size());
        out.resize(out.size() + 2);
        out[static_cast<size_t>(slot)] = HBVHNode{n.box, left, 0};
        st.push_back({n.r, left + 1});
        st.push_back({n.l, left});
    }
    return out;
}

static std::vector<HBVHNode> walkTreeBuild(const std::vector<HBVHNode>& ref, int rounds, int rotSweeps) {
    std::vector<HBVHNode> sweep = rebuildOverLeaves(ref, 2);
    if (rounds <= 0 || sweep.size() < 8) return sweep;
    // The optimisation lowers the BVH2's summed area; the wide tree's, after the collapse, usually
    // with it but not always, and an unconstrained one may deepen the tree (its walk then spills
    // stack entries past the LDS part: the flat stand-in's 13 wide levels became 22, 3.5 % slower).
    // Kept: the first of (free, height-bounded) whose wide tree has a smaller summed area and no
    // more wide levels than the sweep's, then rotated where that lowers the wide area further
    // within the same depth; else the sweep.  (Rotations are not tried on trees the rule rejects:
    // on the flat stand-in they made a rejected tree pass and its shadow walks test 9 % more
    // triangles before an occluder, +1.6 % frame time, profiles/r05_tree_rotation_ab.txt.)
    int dSweep = 0;
    const double aSweep = collapsedArea(sweep, &dSweep);
    for (const bool bounded : {false, true}) {
        std::vector<HBVHNode> opt2 = optimizeOverLeaves(sweep, rounds, bounded);
        int d = 0;
        const double a = collapsedArea(opt2, &d);
        if (a < aSweep && d <= dSweep) {
            std::vector<HBVHNode> rot = rotateForWide(opt2, rotSweeps);
            int dr = 0;
            const double ar = collapsedArea(rot, &dr);
            return ar < a && dr <= dSweep ? rot : opt2;
        }
    }
    return sweep;
}

std::vector<HBVHNode> walkTreeOver(const std::vector<HBVHNode>& ref) {
    const char* walkTree = std::getenv("MOBILERT_WALK_TREE");
    if (walkTree != nullptr && std::atoi(walkTree) == 0) return ref;
    const char* opt = std::getenv("MOBILERT_TREE_OPT");
    const int rounds = opt != nullptr ? std::atoi(opt) : kTreeOptRounds;
    const char* rot = std::getenv("MOBILERT_TREE_ROT");
    const int rotSweeps = rot != nullptr ? std::atoi(rot) : kTreeRotSweeps;
    // Renderers of one scene in one process (a device group's shards, a front end re-creating its
    // renderer, the test suite) share the tree: built once per (reference tree, settings), a few
    // seconds for the conference stand-in.  The key is the whole reference tree's bytes.  A build
    // in flight is shared too: the shards of a device group are created concurrently, and the
    // first to miss builds while the others wait on its future.
    using Tree = std::shared_ptr<const std::vector<HBVHNode>>;
    std::string key(reinterpret_cast<const char*>(ref.data()), ref.size() * sizeof(HBVHNode));
    key.append(reinterpret_cast<const char*>(&rounds), sizeof(rounds));
    key.append(reinterpret_cast<const char*>(&rotSweeps), sizeof(rotSweeps));
    static std::mutex mu;
    static std::unordered_map<std::string, std::shared_future<Tree>> cache;
    static std::deque<std::string> order;  // least recently built first: at most kTreeCacheScenes kept
    std::promise<Tree> mine;
    std::shared_future<Tree> pending;
    {
        std::lock_guard<std::mutex> lock(mu);
        const auto it = cache.find(key);
        if (it != cache.end()) {
            pending = it->second;
        } else {
            cache.emplace(key, mine.get_future().share());
            order.push_back(key);
            while (order.size() > kTreeCacheScenes) {  // (a waiter holds its own copy of the future)
                cache.erase(order.front());
                order.pop_front();
            }
        }
    }
    if (pending.valid()) return *pending.get();  // built, or being built by another thread
    try {
        Tree tree = std::make_shared<const std::vector<HBVHNode>>(walkTreeBuild(ref, rounds, rotSweeps));
        mine.set_value(tree);
        return *tree;
    } catch (...) {
        mine.set_exception(std::current_exception());  // the waiters see the failure too ...
        std::lock_guard<std::mutex> lock(mu);          // ... and a later call builds again
        cache.erase(key);
        order.erase(std::remove(order.begin(), order.end(), key), order.end());
        throw;
    }
}

std::vector<uint32_t> triangleConeWords(const std::vector<HBVHNode>& nodes, const std::vector<HTriangle>& tris) {
    std::vector<uint32_t> out(nodes.size(), kConeNever);
    if (nodes.empty() || tris.empty()) return out;
    // primitive range of every node: leaves hold [indexOffset, +numPrimitives); an inner node
    // the union of its children's (contiguous in BVH order)
    std::vector<std::array<int32_t, 2>> range(nodes.size(), {0, 0});
    std::vector<std::pair<int32_t, bool>> st{{0, false}};
    std::vector<char> seen(nodes.size(), 0);
    while (!st.empty()) {
        const auto [i, post] = st.back();
        st.pop_back();
        const HBVHNode& n = nodes[static_cast<size_t>(i)];
        if (n.numPrimitives > 0 || nodes.size() == 1) {
            range[static_cast<size_t>(i)] = {n.indexOffset, n.indexOffset + n.numPrimitives};
            seen[static_cast<size_t>(i)] = 1;
            continue;
        }
        if (post) {
            const auto& l = range[static_cast<size_t>(n.indexOffset)];
            const auto& r = range[static_cast<size_t>(n.indexOffset) + 1];
            range[static_cast<size_t>(i)] = {std::min(l[0], r[0]), std::max(l[1], r[1])};
            seen[static_cast<size_t>(i)] = 1;
            continue;
        }
        st.push_back({i, true});
        st.push_back({n.indexOffset, false});
        st.push_back({n.indexOffset + 1, false});
    }
    const size_t nn = nodes.size();
    const unsigned hw = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (size_t i = next.fetch_add(64); i < nn; i = next.fetch_add(64)) {
            for (size_t k = i; k < std::min(nn, i + 64); ++k) {
                if (!seen[k]) continue;
                const auto& r = range[k];
                if (r[1] > r[0]) out[k] = coneWord(tris, static_cast<size_t>(r[0]), static_cast<size_t>(r[1]));
            }
        }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < hw; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    return out;
}

// ---- sample tables (Utils.cpp:43-53, Utils.hpp:209-218) ----------------------------------
float haltonSequence(uint32_t index, uint32_t base) {
    float fraction = 1.0F;
    float nextValue = 0.0F;
    const float baseF = static_cast<float>(base);
    while (index > 0) {
        fraction /= baseF;
        nextValue += fraction * static_cast<float>(index % base);
        index = index / base;
    }
    return nextValue;
}

// one entry's cos / sin exactly as the reference evaluates them (std::cos / std::sin of a float:
// libm cosf / sinf; kept out of line so the compiler cannot fold or vectorise the calls)
__attribute__((noinline)) void hemisphereTrig(float r1, float* c, float* s) {
    const float phi = kTwoPi * r1;
    *c = std::cos(phi);
    *s = std::sin(phi);
}

void fillHemisphereTrig(const std::vector<float>& shaderTable, std::vector<float>* out) {
    out->resize(2 * shaderTable.size());
    for (size_t i = 0; i < shaderTable.size(); ++i) hemisphereTrig(shaderTable[i], &(*out)[2 * i], &(*out)[2 * i + 1]);
}

void fillHaltonTable(std::vector<float>* table, uint32_t seed) {
    table->resize(kArraySize);
    for (uint32_t i = 0; i < kArraySize; ++i) (*table)[i] = haltonSequence(i, 2);
    std::mt19937 gen(seed);
    std::shuffle(table->begin(), table->end(), gen);
}

}  // namespace mrt
