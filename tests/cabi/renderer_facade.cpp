// renderer_facade.cpp - builds MobileRT::Renderer from the reference's plugin classes through
// include/mobilert_renderer.hpp, the way app/System_dependent/Native/C_wrapper.cpp:68-210 does
// (scene + camera, pixel sampler by samplesPixel, shader by Config::shader, then
// Renderer(shader, camera, sampler, W, H, spp)), renders one frame per case and writes
// <out>/<case>.bin (the bitmap) and <out>/<case>.txt (getSample, getTotalCastedRays) for
// tests/test_renderer_facade.py to compare with the oracle.
//
// usage: renderer_facade <out dir> <water.obj> <water.mtl> <water.cam> <teapot.obj> <teapot.mtl> <teapot.cam>
#include <cstdio>
#include <fstream>
#include <memory>
#include <string>
#include <vector>

#include "mobilert_renderer.hpp"

namespace {

struct Case {
    const char* name;
    int sceneIndex;  // 0-3 built-in, -1 water OBJ, -2 teapot OBJ
    int shader, spp, accelerator;
};

std::unique_ptr<MobileRT::Sampler> pixelSampler(int spp) {  // C_wrapper.cpp:144-148
    if (spp > 1) return std::unique_ptr<MobileRT::Sampler>(new Components::StaticHaltonSeq());
    return std::unique_ptr<MobileRT::Sampler>(new Components::Constant(0.5F));
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 8) {
        std::fprintf(stderr, "usage: %s <out> <water obj mtl cam> <teapot obj mtl cam>\n", argv[0]);
        return 2;
    }
    const std::string out = argv[1];
    const Case cases[] = {
        {"cornell_whitted", 0, 1, 1, 3},       {"cornell_pathtracer", 0, 2, 2, 3}, {"spheres_whitted", 1, 1, 1, 3},
        {"spheres2_noshadows", 3, 0, 1, 3},    {"cornell2_diffuse", 2, 4, 1, 3},   {"water_pathtracer", -1, 2, 2, 3},
        {"water_depthmap_grid", -1, 3, 1, 2},  {"water_whitted_naive", -1, 1, 1, 1}, {"teapot_whitted", -2, 1, 1, 3},
    };
    const int W = 64, H = 48;
    int failures = 0;
    for (const Case& k : cases) {
        const float ratio = static_cast<float>(W) / static_cast<float>(H);
        MobileRT::Scene scene{};
        std::unique_ptr<MobileRT::Camera> camera;
        MobileRT::Vec3 maxDist{1.0F, 1.0F, 1.0F};
        switch (k.sceneIndex) {  // C_wrapper.cpp:76-141
            case 0: scene = cornellBox_Scene(std::move(scene)); camera = cornellBox_Cam(ratio); break;
            case 1: scene = spheres_Scene(std::move(scene)); camera = spheres_Cam(ratio); maxDist = {8, 8, 8}; break;
            case 2: scene = cornellBox2_Scene(std::move(scene)); camera = cornellBox_Cam(ratio); break;
            case 3: scene = spheres2_Scene(std::move(scene)); camera = spheres2_Cam(ratio); maxDist = {8, 8, 8}; break;
            default: {
                const int base = k.sceneIndex == -1 ? 2 : 5;
                std::ifstream ifObj{argv[base]};
                std::ifstream ifMtl{argv[base + 1]};
                Components::OBJLoader objLoader{ifObj, ifMtl};
                if (!objLoader.isProcessed()) return 1;
                std::unordered_map<std::string, MobileRT::Texture> texturesCache{};
                const bool built = objLoader.fillScene(
                    &scene, []() { return std::unique_ptr<MobileRT::Sampler>(new Components::StaticHaltonSeq()); },
                    argv[base], texturesCache);
                if (!built) return 1;
                std::ifstream ifCamera{argv[base + 2]};
                std::istream iCam{ifCamera.rdbuf()};
                camera = Components::CameraFactory().loadFromFile(iCam, ratio);
            }
        }
        std::unique_ptr<MobileRT::Shader> shader;
        const auto acc = MobileRT::Shader::Accelerator(k.accelerator);
        switch (k.shader) {  // C_wrapper.cpp:154-193
            case 1: shader.reset(new Components::Whitted(std::move(scene), 1, acc)); break;
            case 2: {
                std::unique_ptr<MobileRT::Sampler> rr{new Components::StaticHaltonSeq()};
                shader.reset(new Components::PathTracer(std::move(scene), std::move(rr), 1, acc));
                break;
            }
            case 3: shader.reset(new Components::DepthMap(std::move(scene), maxDist, acc)); break;
            case 4: shader.reset(new Components::DiffuseMaterial(std::move(scene), acc)); break;
            default: shader.reset(new Components::NoShadows(std::move(scene), 1, acc)); break;
        }
        try {
            MobileRT::Renderer renderer{std::move(shader), std::move(camera), pixelSampler(k.spp), W, H, k.spp};
            std::vector<std::int32_t> bitmap(static_cast<size_t>(W) * H, 0);
            renderer.renderFrame(bitmap.data(), 3);
            std::ofstream(out + "/" + k.name + ".bin", std::ios::binary)
                .write(reinterpret_cast<const char*>(bitmap.data()), static_cast<std::streamsize>(bitmap.size() * 4));
            std::ofstream(out + "/" + k.name + ".txt") << renderer.getSample() << " " << renderer.getTotalCastedRays() << "\n";
            std::printf("case %s: sample %d rays %llu\n", k.name, renderer.getSample(),
                        static_cast<unsigned long long>(renderer.getTotalCastedRays()));
        } catch (const std::exception& e) {
            std::printf("case %s: error %s\n", k.name, e.what());
            ++failures;
        }
    }
    return failures == 0 ? 0 : 1;
}
