// mobilert_renderer.hpp - the reference's in-process C++ plugin surface over the MI355X path.
//
// app/MobileRT/Renderer.hpp:41-63 builds a renderer from the plugins a front end assembles
// (app/System_dependent/Native/C_wrapper.cpp:68-210):
//
//     Renderer(std::unique_ptr<Shader>, std::unique_ptr<Camera>, std::unique_ptr<Sampler>,
//              int32_t width, int32_t height, int32_t samplesPixel);
//     void renderFrame(int32_t *bitmap, int32_t numThreads);  stopRender();
//     int32_t getSample() const;  uint64_t getTotalCastedRays() const;
//
// This header keeps those names, constructors and meanings for the concrete plugins the native
// path uses - shaders Whitted / PathTracer / DepthMap / DiffuseMaterial / NoShadows
// (app/Components/Shaders), cameras Perspective / Orthographic (app/Components/Cameras), samplers
// Constant / StaticHaltonSeq (app/Components/Samplers), the built-in scenes and their cameras
// (app/Scenes/Scenes.hpp), OBJLoader and CameraFactory (app/Components/Loaders) - so that code
// written against the reference's classes, like C_wrapper.cpp's work_thread, compiles against this
// header unchanged apart from the include lines.  The plugins are descriptions: the Renderer
// hands them to libmobilert_amd.so (include/mobilert_amd.h: mrt_create_from_memory,
// mrt_set_camera, mrt_set_pixel_sampler, mrt_set_max_point), which builds the scene, the BVH and
// the device buffers once and renders every frame with the HIP kernels.
//
// Differences to the reference, all forced by the GPU path or by determinism (DESIGN.md section
// 4): every sampler draw comes from the deterministic tables (a PathTracer's Russian-roulette
// sampler and an area light's sampler are accepted but not called); Sampler::getSample on the host
// returns the same Halton sequence but is not what the kernels read; numThreads is ignored; the
// camera a CameraFactory loads is parsed by the library at the Renderer's aspect ratio
// (width / height, as C_wrapper.cpp passes); vectors are MobileRT::Vec3 (constructible from any
// type with x, y, z, e.g. glm::vec3).
#ifndef MOBILERT_RENDERER_HPP
#define MOBILERT_RENDERER_HPP

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <istream>
#include <iterator>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "mobilert_amd.h"

namespace MobileRT {

struct Vec3 {
    float x{}, y{}, z{};
    Vec3() = default;
    Vec3(float vx, float vy, float vz) : x(vx), y(vy), z(vz) {}
    template <class V, class = decltype(std::declval<const V&>().z)>
    Vec3(const V& v) : x(static_cast<float>(v.x)), y(static_cast<float>(v.y)), z(static_cast<float>(v.z)) {}
};

// Texture.hpp: the value type of OBJLoader::fillScene's texture cache (textures are decoded by
// the library; the cache is accepted for signature compatibility).
struct Texture {};

// Scene.hpp: what a Shader's accelerators are built from - here a built-in scene of Scenes.cpp
// (builtin 0-3) or an OBJ / MTL definition filled by OBJLoader (builtin -1).
class Scene {
public:
    std::int32_t builtin{-1};
    std::string obj, mtl, objPath;
    std::vector<std::pair<std::string, std::string>> textures;  // file name -> bytes (map_Kd)
};

// Sampler.hpp:13-64
class Sampler {
public:
    virtual ~Sampler() = default;
    virtual float getSample(std::uint32_t sample) = 0;
    float getSample() { return getSample(0); }  // Sampler.cpp:44-46
    virtual void resetSampling() {}
    // the device's pixel sampler: 0 Constant(value), 1 StaticHaltonSeq (mrt_set_pixel_sampler)
    virtual std::int32_t deviceKind() const = 0;
    virtual float deviceValue() const { return 0.5F; }
};

// Camera.hpp:16-71: position, look-at and up (Camera.cpp:14-19 derives direction, right, up')
class Camera {
public:
    virtual ~Camera() = default;
    // 0 Perspective (a, b = hFov, vFov in degrees), 1 Orthographic (a, b = sizeH, sizeV),
    // 2 a camera definition parsed by the library (CameraFactory)
    std::int32_t kind{0};
    Vec3 position, lookAt, up;
    float a{}, b{};
    std::string definition;

protected:
    Camera() = default;
};

// Shader.hpp:20-24 and the constructor arguments every shader shares
class Shader {
public:
    enum Accelerator { ACC_NAIVE = 1, ACC_REGULAR_GRID, ACC_BVH };
    virtual ~Shader() = default;
    const Scene& scene() const { return scene_; }
    std::int32_t samplesLight() const { return samplesLight_; }
    Accelerator accelerator() const { return accelerator_; }
    // Config::shader's value (C_wrapper.cpp:154-193): 0 NoShadows, 1 Whitted, 2 PathTracer,
    // 3 DepthMap, 4 DiffuseMaterial
    virtual std::int32_t configId() const = 0;
    const Vec3* maxPoint() const { return hasMaxPoint_ ? &maxPoint_ : nullptr; }

protected:
    Shader(Scene scene, std::int32_t samplesLight, Accelerator accelerator)
        : scene_(std::move(scene)), samplesLight_(samplesLight), accelerator_(accelerator) {}
    Scene scene_;
    std::int32_t samplesLight_;
    Accelerator accelerator_;
    Vec3 maxPoint_;
    bool hasMaxPoint_ = false;
};

// Renderer.hpp:41-63 over the C-ABI (one mrt_renderer per Renderer, scene uploaded once).
class Renderer final {
public:
    Renderer() = delete;
    Renderer(std::unique_ptr<Shader> shader, std::unique_ptr<Camera> camera, std::unique_ptr<Sampler> samplerPixel,
             std::int32_t width, std::int32_t height, std::int32_t samplesPixel)
        : shader_(std::move(shader)), camera_(std::move(camera)), sampler_(std::move(samplerPixel)) {
        if (!shader_ || !camera_ || !sampler_) throw std::invalid_argument("Renderer: null plugin");
        const Scene& sc = shader_->scene();
        mrt_config c{};
        c.width = width;
        c.height = height;
        c.threads = 1;
        c.shader = shader_->configId();
        c.sceneIndex = sc.builtin;
        c.samplesPixel = samplesPixel;
        c.samplesLight = shader_->samplesLight();
        c.repeats = 1;
        c.accelerator = static_cast<std::int32_t>(shader_->accelerator());
        c.objFilePath = sc.objPath.c_str();
        c.mtlFilePath = "";
        c.camFilePath = "";
        const char* md = std::getenv("MOBILERT_MAX_DEPTH");  // RayDepthMax (Constants.hpp:45); 0 -> 6
        c.maxDepth = md != nullptr ? std::atoi(md) : 0;
        c.rankCount = 1;
        c.device = -1;
        // MOBILERT_DEVICES=0,1,...: the frame sharded over these GPUs (mrt_config.devices; the
        // reference's renderFrame spreads a frame over its workers, Renderer.cpp:62-82)
        // (the same rules and message as the library's own parser, mrt::parseDeviceList: every item a
        // whole non-negative decimal ordinal)
        std::vector<std::int32_t> devices;
        const char* dl = std::getenv("MOBILERT_DEVICES");
        if (dl != nullptr && *dl != '\0') {
            std::string item;
            for (const char* q = dl;; ++q) {
                if (*q == '\0' && item.empty() && q != dl) break;  // a trailing comma ends the list
                if (*q == ',' || *q == '\0') {
                    char* end = nullptr;
                    const long v = std::strtol(item.c_str(), &end, 10);
                    if (item.empty() || end != item.c_str() + item.size() || v < 0 || v > 0x7fffffffL)
                        throw std::runtime_error("MOBILERT_DEVICES: bad ordinal '" + item + "'");
                    devices.push_back(static_cast<std::int32_t>(v));
                    item.clear();
                    if (*q == '\0') break;
                } else {
                    item.push_back(*q);
                }
            }
        }
        if (devices.size() > 1) {
            c.devices = devices.data();
            c.deviceCount = static_cast<std::int32_t>(devices.size());
        }
        c.cull = 3;         // exact for every input
        c.progressive = 1;  // the bitmap and getSample() advance sample by sample (Renderer.cpp:53-88)
        // a camera given as parameters is set after creation; a loaded definition is parsed there
        static const char kPlaceholderCam[] = "t perspective\np 0 0 0\nl 0 0 1\nu 0 1 0\nf 45 45\n";
        const std::string cam = camera_->kind == 2 ? camera_->definition : std::string(kPlaceholderCam);
        std::vector<mrt_blob> blobs;
        for (const auto& t : sc.textures)
            blobs.push_back(mrt_blob{t.first.c_str(), reinterpret_cast<const std::uint8_t*>(t.second.data()),
                                     static_cast<std::int64_t>(t.second.size())});
        mrt_renderer* r = nullptr;
        const bool builtin = sc.builtin >= 0 && sc.builtin <= 3;
        const int rc = builtin ? mrt_create(&c, &r)
                               : mrt_create_from_memory(&c, sc.obj.data(), static_cast<std::int64_t>(sc.obj.size()),
                                                        sc.mtl.data(), static_cast<std::int64_t>(sc.mtl.size()),
                                                        cam.data(), static_cast<std::int64_t>(cam.size()), blobs.data(),
                                                        static_cast<std::int32_t>(blobs.size()), &r);
        if (rc != 0) throw std::runtime_error(mrt_last_error());
        h_ = r;
        if (camera_->kind != 2) {
            const float p[3] = {camera_->position.x, camera_->position.y, camera_->position.z};
            const float l[3] = {camera_->lookAt.x, camera_->lookAt.y, camera_->lookAt.z};
            const float u[3] = {camera_->up.x, camera_->up.y, camera_->up.z};
            check(mrt_set_camera(h_, camera_->kind, p, l, u, camera_->a, camera_->b));
        }
        check(mrt_set_pixel_sampler(h_, sampler_->deviceKind(), sampler_->deviceValue()));
        if (const Vec3* m = shader_->maxPoint()) {
            const float mp[3] = {m->x, m->y, m->z};
            check(mrt_set_max_point(h_, mp));
        }
    }
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;
    ~Renderer() {
        if (h_ != nullptr) mrt_destroy(h_);
    }
    // Renderer.cpp:53-88: every sample of the frame into bitmap (width * height ABGR int32)
    void renderFrame(std::int32_t* bitmap, std::int32_t numThreads) {
        (void)numThreads;
        check(mrt_render_frame(h_, bitmap));
    }
    void stopRender() { (void)mrt_stop_render(h_); }  // Renderer.cpp:93-99
    std::int32_t getSample() const { return mrt_get_sample(h_); }
    std::uint64_t getTotalCastedRays() const { return mrt_get_total_casted_rays(h_); }
    mrt_renderer* handle() const { return h_; }

    std::unique_ptr<Shader> shader_;
    std::unique_ptr<Camera> camera_;

private:
    static void check(int rc) {
        if (rc != 0) throw std::runtime_error(mrt_last_error());
    }
    std::unique_ptr<Sampler> sampler_;
    mrt_renderer* h_ = nullptr;
};

}  // namespace MobileRT

namespace Components {

// Constant.cpp:9-11
class Constant final : public ::MobileRT::Sampler {
public:
    Constant() = delete;
    explicit Constant(float value) : value_(value) {}
    float getSample(std::uint32_t) override { return value_; }
    std::int32_t deviceKind() const override { return 0; }
    float deviceValue() const override { return value_; }

private:
    float value_;
};

// StaticHaltonSeq.cpp:7-22 (here unshuffled: the device draws from the fixed-seed tables)
class StaticHaltonSeq final : public ::MobileRT::Sampler {
public:
    StaticHaltonSeq() = default;
    StaticHaltonSeq(std::uint32_t, std::uint32_t, std::uint32_t) {}
    float getSample(std::uint32_t) override {  // Utils.cpp:43-53 haltonSequence(i, 2)
        std::uint32_t index = cursor_.fetch_add(1) & 0xFFFFFu;
        float fraction = 1.0F, result = 0.0F;
        while (index > 0) {
            fraction /= 2.0F;
            result += fraction * static_cast<float>(index % 2);
            index = index / 2;
        }
        return result;
    }
    std::int32_t deviceKind() const override { return 1; }

private:
    std::atomic<std::uint32_t> cursor_{0};
};

// Perspective.cpp:8-14 (fovs in degrees)
class Perspective final : public ::MobileRT::Camera {
public:
    Perspective() = delete;
    Perspective(const ::MobileRT::Vec3& position, const ::MobileRT::Vec3& lookAt, const ::MobileRT::Vec3& up,
                float hFov, float vFov) {
        kind = 0;
        this->position = position;
        this->lookAt = lookAt;
        this->up = up;
        a = hFov;
        b = vFov;
    }
};

// Orthographic.cpp:7-13
class Orthographic final : public ::MobileRT::Camera {
public:
    Orthographic() = delete;
    Orthographic(const ::MobileRT::Vec3& position, const ::MobileRT::Vec3& lookAt, const ::MobileRT::Vec3& up,
                 float sizeH, float sizeV) {
        kind = 1;
        this->position = position;
        this->lookAt = lookAt;
        this->up = up;
        a = sizeH;
        b = sizeV;
    }
};

// CameraFactory.cpp + PerspectiveLoader.cpp: the .cam definition, parsed by the library
class LoadedCamera final : public ::MobileRT::Camera {
public:
    explicit LoadedCamera(std::string text) {
        kind = 2;
        definition = std::move(text);
    }
};

class CameraFactory {
public:
    std::unique_ptr<::MobileRT::Camera> loadFromFile(std::istream& isCam, float aspectRatio) const {
        (void)aspectRatio;  // the library applies width / height (PerspectiveLoader.cpp:59)
        std::string text{std::istreambuf_iterator<char>(isCam), std::istreambuf_iterator<char>()};
        return std::unique_ptr<::MobileRT::Camera>(new LoadedCamera(std::move(text)));
    }
};

// OBJLoader.hpp:18-80: the OBJ / MTL text; the library parses it when the Renderer is built
// (tinyobjloader v1.0.7's rules, mrt_scene.cpp), and reads map_Kd textures named in the MTL from
// the OBJ file's directory here.
class OBJLoader final {
public:
    OBJLoader() = delete;
    OBJLoader(std::istream& isObj, std::istream& isMtl)
        : obj_{std::istreambuf_iterator<char>(isObj), std::istreambuf_iterator<char>()},
          mtl_{std::istreambuf_iterator<char>(isMtl), std::istreambuf_iterator<char>()} {}
    bool isProcessed() const { return !obj_.empty(); }
    bool fillScene(::MobileRT::Scene* scene, std::function<std::unique_ptr<::MobileRT::Sampler>()> lambda,
                   std::string filePath, std::unordered_map<std::string, ::MobileRT::Texture> texturesCache) {
        (void)lambda;
        (void)texturesCache;
        if (scene == nullptr || obj_.empty()) return false;
        scene->builtin = -1;
        scene->obj = obj_;
        scene->mtl = mtl_;
        scene->objPath = filePath;
        const std::string dir = filePath.substr(0, filePath.find_last_of('/') + 1);
        std::istringstream mtl(mtl_);
        std::string line;
        while (std::getline(mtl, line)) {
            std::istringstream ls(line);
            std::string key, name;
            if (!(ls >> key) || key != "map_Kd" || !(ls >> name)) continue;
            std::ifstream f(dir + name, std::ios::binary);
            if (!f) continue;
            std::string bytes{std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>()};
            scene->textures.emplace_back(name.substr(name.find_last_of('/') + 1), std::move(bytes));
        }
        return true;
    }

private:
    std::string obj_, mtl_;
};

// The shaders (app/Components/Shaders/*.hpp), with the reference's constructors
class Whitted final : public ::MobileRT::Shader {
public:
    Whitted(::MobileRT::Scene scene, std::int32_t samplesLight, Accelerator accelerator)
        : Shader(std::move(scene), samplesLight, accelerator) {}
    std::int32_t configId() const override { return 1; }
};

class PathTracer final : public ::MobileRT::Shader {
public:
    PathTracer(::MobileRT::Scene scene, std::unique_ptr<::MobileRT::Sampler> samplerRussianRoulette,
               std::int32_t samplesLight, Accelerator accelerator)
        : Shader(std::move(scene), samplesLight, accelerator), samplerRussianRoulette_(std::move(samplerRussianRoulette)) {}
    std::int32_t configId() const override { return 2; }

private:
    std::unique_ptr<::MobileRT::Sampler> samplerRussianRoulette_;
};

class DepthMap final : public ::MobileRT::Shader {
public:
    DepthMap(::MobileRT::Scene scene, const ::MobileRT::Vec3& maxPoint, Accelerator accelerator)
        : Shader(std::move(scene), 1, accelerator) {
        maxPoint_ = maxPoint;
        hasMaxPoint_ = true;
    }
    std::int32_t configId() const override { return 3; }
};

class DiffuseMaterial final : public ::MobileRT::Shader {
public:
    DiffuseMaterial(::MobileRT::Scene scene, Accelerator accelerator) : Shader(std::move(scene), 1, accelerator) {}
    std::int32_t configId() const override { return 4; }
};

class NoShadows final : public ::MobileRT::Shader {
public:
    NoShadows(::MobileRT::Scene scene, std::int32_t samplesLight, Accelerator accelerator)
        : Shader(std::move(scene), samplesLight, accelerator) {}
    std::int32_t configId() const override { return 0; }
};

}  // namespace Components

// Scenes.hpp: the built-in scenes (the library builds their geometry, Scenes.cpp:63-302) and
// their cameras (Scenes.cpp:139-150, 251-262, 291-302)
inline ::MobileRT::Scene cornellBox_Scene(::MobileRT::Scene scene) { scene.builtin = 0; return scene; }
inline ::MobileRT::Scene spheres_Scene(::MobileRT::Scene scene) { scene.builtin = 1; return scene; }
inline ::MobileRT::Scene cornellBox2_Scene(::MobileRT::Scene scene) { scene.builtin = 2; return scene; }
inline ::MobileRT::Scene spheres2_Scene(::MobileRT::Scene scene) { scene.builtin = 3; return scene; }
inline std::unique_ptr<::MobileRT::Camera> cornellBox_Cam(float ratio) {
    return std::unique_ptr<::MobileRT::Camera>(new ::Components::Perspective(
        ::MobileRT::Vec3{0.0F, 0.0F, -3.4F}, ::MobileRT::Vec3{0.0F, 0.0F, 1.0F}, ::MobileRT::Vec3{0.0F, 1.0F, 0.0F},
        45.0F * ratio, 45.0F));
}
inline std::unique_ptr<::MobileRT::Camera> cornellBox2_Cam(float ratio) { return cornellBox_Cam(ratio); }
inline std::unique_ptr<::MobileRT::Camera> spheres_Cam(float ratio) {
    return std::unique_ptr<::MobileRT::Camera>(new ::Components::Orthographic(
        ::MobileRT::Vec3{0.0F, 1.0F, -10.0F}, ::MobileRT::Vec3{0.0F, 1.0F, 7.0F}, ::MobileRT::Vec3{0.0F, 1.0F, 0.0F},
        10.0F * ratio, 10.0F));
}
inline std::unique_ptr<::MobileRT::Camera> spheres2_Cam(float ratio) {
    return std::unique_ptr<::MobileRT::Camera>(new ::Components::Perspective(
        ::MobileRT::Vec3{0.0F, 0.5F, 1.0F}, ::MobileRT::Vec3{0.0F, 0.0F, 7.0F}, ::MobileRT::Vec3{0.0F, 1.0F, 0.0F},
        60.0F * ratio, 60.0F));
}

#endif  // MOBILERT_RENDERER_HPP
