// mobilert_amd.hpp - the reference's desktop C-ABI, unchanged, over the MI355X path.
//
// app/System_dependent/Native/C_wrapper.h:12-20 declares
//     extern "C" void RayTrace(::MobileRT::Config &config, bool async);
//     extern "C" void stopRender();
// with MobileRT::Config from app/MobileRT/Config.hpp:12-83.  This header re-declares the same
// struct (same members, same order, same types) so a front end built against the reference
// header links against libmobilert_amd.so unchanged.  GPU-only knobs come from environment
// variables, see INTEGRATION.md: MOBILERT_MAX_DEPTH (RayDepthMax), MOBILERT_DEVICE (the one GPU to
// render on) and MOBILERT_DEVICES ("0,1,..": a device group - the frame's screen-tile shards spread
// over these GPUs from one process, as renderFrame spreads it over its workers, Renderer.cpp:62-82).
#ifndef MOBILERT_AMD_HPP
#define MOBILERT_AMD_HPP

#include <cstdint>
#include <string>
#include <vector>

#include "mobilert_amd.h"

namespace MobileRT {
struct Config {
public:
    ::std::vector<::std::int32_t> bitmap;
    ::std::string objFilePath;
    ::std::string mtlFilePath;
    ::std::string camFilePath;
    ::std::int32_t width;
    ::std::int32_t height;
    ::std::int32_t threads;
    ::std::int32_t shader;
    ::std::int32_t sceneIndex;
    ::std::int32_t samplesPixel;
    ::std::int32_t samplesLight;
    ::std::int32_t repeats;
    ::std::int32_t accelerator;
    bool printStdOut;
};
}  // namespace MobileRT

extern "C" void RayTrace(::MobileRT::Config &config, bool async);
extern "C" void stopRender();

#endif  // MOBILERT_AMD_HPP
