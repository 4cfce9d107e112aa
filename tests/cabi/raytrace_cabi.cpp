// raytrace_cabi.cpp - drives the reference's desktop C-ABI, RayTrace(Config&, bool) and
// stopRender() (app/System_dependent/Native/C_wrapper.h:12-20), from C++ through
// include/mobilert_amd.hpp, the way the reference's engine tests do
// (app/Unit_Testing/engine/{Shader,Accelerator,Camera}TestEngine.cpp): a 30x30 Config with 3
// threads, 1 sample per pixel and light, one repeat, stdout summary on; the bitmap is uniform
// before and not uniform after.  Every bitmap is written to <out>/<case>.bin for
// tests/test_cabi_cpp.py to compare with the oracle.  Then an asynchronous render is stopped
// through stopRender() while it runs.
//
// usage: raytrace_cabi <out dir> <CornellBox-Water.obj> <.mtl> <.cam>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "mobilert_amd.hpp"

namespace {

struct Case {
    const char* name;
    int32_t sceneIndex, shader, accelerator;
    bool obj;
};

bool uniform(const std::vector<int32_t>& b) {
    return std::all_of(b.begin() + 1, b.end(), [&](int32_t v) { return v == b.front(); });
}

// ShaderTestEngine.cpp:10-24 (SetUp)
MobileRT::Config setUp() {
    MobileRT::Config config{};
    config.width = 30;
    config.height = 30;
    config.threads = 3;
    config.sceneIndex = 1;
    config.samplesPixel = 1;
    config.samplesLight = 1;
    config.repeats = 1;
    config.printStdOut = true;
    config.objFilePath = std::string{""};
    config.mtlFilePath = std::string{""};
    config.camFilePath = std::string{""};
    config.bitmap = std::vector<int32_t>(static_cast<size_t>(config.width) * static_cast<size_t>(config.height));
    return config;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s <out dir> <obj> <mtl> <cam>\n", argv[0]);
        return 2;
    }
    const std::string out = argv[1];
    const Case cases[] = {
        {"noshadows_water", -1, 0, 3, true},     // ShaderTestEngine testRenderSceneWithNoShadows
        {"whitted_water", -1, 1, 3, true},       // testRenderSceneWithWhitted
        {"pathtracer_water", -1, 2, 3, true},    // testRenderSceneWithPathTracing
        {"depthmap_water", -1, 3, 3, true},      // testRenderSceneWithDepthMap
        {"diffuse_water", -1, 4, 3, true},       // testRenderSceneWithDiffuse
        {"naive_water", -1, 1, 1, true},         // AcceleratorTestEngine testRenderSceneWithNaive
        {"grid_water", -1, 1, 2, true},          // testRenderSceneWithRegularGrid
        {"bvh_water", -1, 1, 3, true},           // testRenderSceneWithBVH
        {"orthographic_spheres", 1, 1, 3, false},  // CameraTestEngine testRenderSceneWithOrthographic
        {"perspective_cornell", 0, 1, 3, false},   // testRenderSceneWithPerspective
        {"pathtracer_cornell", 0, 2, 3, false},
    };
    int failures = 0;
    for (const Case& c : cases) {
        MobileRT::Config config = setUp();
        config.sceneIndex = c.sceneIndex;
        config.shader = c.shader;
        config.accelerator = c.accelerator;
        if (c.obj) {
            config.objFilePath = std::string{argv[2]};
            config.mtlFilePath = std::string{argv[3]};
            config.camFilePath = std::string{argv[4]};
        }
        if (!uniform(config.bitmap)) ++failures;
        RayTrace(config, false);
        const bool ok = !uniform(config.bitmap);
        if (!ok) ++failures;
        std::printf("case %s: %s\n", c.name, ok ? "rendered" : "UNIFORM BITMAP");
        std::ofstream f(out + "/" + c.name + ".bin", std::ios::binary);
        f.write(reinterpret_cast<const char*>(config.bitmap.data()),
                static_cast<std::streamsize>(config.bitmap.size() * sizeof(int32_t)));
    }
    // asynchronous render (C_wrapper.cpp:268-282: a detached thread) stopped by stopRender()
    // while it runs: a progressive frame of 256 samples renders a few, then stops between samples
    {
        MobileRT::Config config = setUp();
        config.width = config.height = 512;
        config.sceneIndex = 0;
        config.shader = 2;
        config.accelerator = 3;
        config.samplesPixel = 256;
        config.printStdOut = false;
        config.bitmap = std::vector<int32_t>(512 * 512);
        RayTrace(config, true);
        const auto t0 = std::chrono::steady_clock::now();
        while (uniform(config.bitmap) && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(60))
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        stopRender();
        // the caller keeps config alive until the render thread has left (it touches config.bitmap
        // after each sample): wait until the bitmap stays the same for a while
        std::vector<int32_t> last = config.bitmap;
        int stable = 0;
        for (int i = 0; i < 600 && stable < 50; ++i) {
            std::this_thread::sleep_for(std::chrono::milliseconds(10));
            stable = (config.bitmap == last) ? stable + 1 : 0;
            last = config.bitmap;
        }
        const bool ok = !uniform(config.bitmap) && stable >= 50;
        if (!ok) ++failures;
        std::printf("case async_stop: %s\n", ok ? "rendered and stopped" : "FAILED");
        std::ofstream f(out + "/async_stop.bin", std::ios::binary);
        f.write(reinterpret_cast<const char*>(config.bitmap.data()),
                static_cast<std::streamsize>(config.bitmap.size() * sizeof(int32_t)));
    }
    // let the detached render thread release the renderer before the process exits
    std::this_thread::sleep_for(std::chrono::seconds(1));
    std::printf("failures %d\n", failures);
    return failures == 0 ? 0 : 1;
}
