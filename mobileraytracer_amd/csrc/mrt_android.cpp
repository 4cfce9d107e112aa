// mrt_android.cpp - the Android front end's native session (include/mobilert_android.h).
//
// The state machine and ownership of app/System_dependent/Android_JNI/JNI_layer.cpp, over the
// library's C-ABI: one renderer, the scene files handed over by readFile, the render thread
// started by rtRenderIntoBitmap, and the getters the Kotlin RenderTask polls.  The reference keeps
// renderer_ in a unique_ptr that rtInitialize may reset while a render thread still uses it; here
// the render thread holds its own reference (a shared_ptr), so a re-initialize cannot free the
// renderer under a running frame.  Everything else follows the reference, including its quirks
// (rtStopRender's wait returns at once when a renderer exists, :440-452; the fps counter's first
// interval runs from the clock's epoch, :391-404).
#include "mobilert_amd.h"
#include "mobilert_android.h"
#include "mrt_scene.hpp"

#include <atomic>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

std::mutex gMutex;                    // guards the renderer and the cached files (JNI_layer.cpp:64)
std::condition_variable gRendered;    // :79
std::condition_variable gIdle;        // a render thread ended (gActive dropped)
int32_t gActive = 0;                  // render threads still running (guarded by gMutex)
std::atomic<int32_t> gState{MRT_STATE_IDLE};
std::atomic<bool> gFinished{true};    // finishedRendering_ (:84)
std::atomic<float> gFps{0.0F};
std::atomic<int64_t> gTimeRenderer{0};
std::atomic<int32_t> gNumLights{0};
std::shared_ptr<mrt_renderer> gRenderer;
std::string gObj, gMtl, gCam;                  // objDefinition_ / mtlDefinition_ / camDefinition_
std::map<std::string, std::string> gTextures;  // texturesCache_ (by file name)

void updateFps() {  // JNI_layer.cpp:391-404
    static int32_t frame = 0;
    static std::chrono::steady_clock::time_point timebase{};
    ++frame;
    const auto now = std::chrono::steady_clock::now();
    const long long elapsed = std::chrono::duration_cast<std::chrono::milliseconds>(now - timebase).count();
    gFps = (static_cast<float>(frame) * 1000.0F) / static_cast<float>(elapsed);
    if (elapsed > 1000) {
        timebase = now;
        frame = 0;
    }
}

// handleException (:114-126): the Java side gets an exception; the state resets
void onError() {
    gState = MRT_STATE_IDLE;
    gFinished = true;
}

std::shared_ptr<mrt_renderer> current() {
    std::lock_guard<std::mutex> lock(gMutex);
    return gRenderer;
}

// Cancels the render in flight and waits for its thread to end (the lock is released while
// waiting): the renderer and the caller's pixels may be replaced or freed only after that, since
// the thread's last mrt_render_frame writes the pixels until it returns.
void stopAndWait(std::unique_lock<std::mutex>& lock) {
    if (gActive == 0) return;
    if (gRenderer != nullptr) mrt_stop_render(gRenderer.get());
    gIdle.wait(lock, [] { return gActive == 0; });
}

}  // namespace

extern "C" {

void mrt_android_read_file(const char* path, const uint8_t* bytes, int64_t size) {
    const std::string p = path != nullptr ? path : "";
    const size_t dot = p.find_last_of('.');
    const std::string ext = dot == std::string::npos ? std::string() : p.substr(dot);
    const std::string content(reinterpret_cast<const char*>(bytes), static_cast<size_t>(size > 0 ? size : 0));
    std::lock_guard<std::mutex> lock(gMutex);
    if (ext == ".obj") {
        gObj = content;
    } else if (ext == ".mtl") {
        gMtl = content;
    } else if (ext == ".cam") {
        gCam = content;
    } else {  // a texture: OBJLoader::getTextureFromCache keyed by the file name (:1036-1045)
        gTextures[p.substr(p.find_last_of('/') + 1)] = content;
    }
}

int32_t mrt_android_initialize(const mrt_android_config* config) {
    try {
        std::unique_lock<std::mutex> lock(gMutex);
        stopAndWait(lock);
        gRenderer.reset();
        mrt_config c{};
        c.width = config->width;
        c.height = config->height;
        c.threads = 1;
        c.shader = config->shader;
        c.sceneIndex = config->scene;
        c.samplesPixel = config->samplesPixel;
        c.samplesLight = config->samplesLight;
        c.repeats = 1;
        c.accelerator = config->accelerator;
        c.objFilePath = config->objFilePath != nullptr ? config->objFilePath : "";
        c.mtlFilePath = "";
        c.camFilePath = "";
        c.rankCount = 1;
        c.device = -1;
        c.cull = 3;  // exact for every input
        c.progressive = 1;  // the bitmap fills sample by sample while RenderTask polls it
        // MOBILERT_DEVICES=0,1,...: the frame sharded over these GPUs (a device group)
        const std::vector<int32_t> devices = mrt::parseDeviceList(std::getenv("MOBILERT_DEVICES"));
        if (devices.size() > 1) {
            c.devices = devices.data();
            c.deviceCount = static_cast<int32_t>(devices.size());
        }
        const bool builtin = config->scene >= 0 && config->scene <= 3;
        mrt_renderer* r = nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        int rc;
        if (builtin) {  // from memory too, so the renderer keeps its host scene for the GL preview
            rc = mrt_create_from_memory(&c, nullptr, 0, nullptr, 0, nullptr, 0, nullptr, 0, &r);
        } else {
            std::vector<std::string> names;
            std::vector<mrt_blob> blobs;
            names.reserve(gTextures.size());
            for (const auto& t : gTextures) {
                names.push_back(t.first);
                blobs.push_back(mrt_blob{names.back().c_str(), reinterpret_cast<const uint8_t*>(t.second.data()),
                                         static_cast<int64_t>(t.second.size())});
            }
            const std::string obj = std::move(gObj), mtl = std::move(gMtl), cam = std::move(gCam);
            gObj.clear();  // the definitions are consumed by this call (:570-581, :589)
            gMtl.clear();
            gCam.clear();
            rc = mrt_create_from_memory(&c, obj.data(), static_cast<int64_t>(obj.size()), mtl.data(),
                                        static_cast<int64_t>(mtl.size()), cam.data(), static_cast<int64_t>(cam.size()),
                                        blobs.data(), static_cast<int32_t>(blobs.size()), &r);
            gTextures.clear();
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (rc != 0) throw std::runtime_error(mrt_last_error());
        gRenderer = std::shared_ptr<mrt_renderer>(r, mrt_destroy);
        mrt_scene_info info{};
        mrt_get_scene_info(r, &info);
        gNumLights = static_cast<int32_t>(info.lights);
        gTimeRenderer = std::chrono::duration_cast<std::chrono::milliseconds>(t1 - t0).count();
        return static_cast<int32_t>(info.triangles + info.spheres + info.planes);
    } catch (const std::bad_alloc&) {
        onError();
        return -1;
    } catch (const std::exception&) {
        onError();
        return -2;
    } catch (...) {
        onError();
        return -3;
    }
}

void mrt_android_render_into_bitmap_cb(int32_t* pixels, int32_t nThreads, mrt_android_done_fn done, void* user) {
    (void)nThreads;  // Renderer::renderFrame's thread count: the GPU path does not use it
    std::shared_ptr<mrt_renderer> r;
    {
        std::lock_guard<std::mutex> lock(gMutex);
        r = gRenderer;
        ++gActive;  // before the thread starts: an initialize / reset right after this call waits for it
    }
    auto body = [r, pixels, done, user] {  // detached render thread (:883-889)
        int32_t rep = 1;
        while (gState == MRT_STATE_BUSY && rep > 0) {
            if (r != nullptr) (void)mrt_render_frame(r.get(), pixels);
            updateFps();
            rep--;
        }
        // the last frame has returned: the caller may release the pixels now (the reference unlocks
        // the Android bitmap here, in the render thread, :850-854)
        if (done != nullptr) done(user);
        gFinished = true;
        gRendered.notify_all();
        {
            std::lock_guard<std::mutex> lock(gMutex);
            if (gState != MRT_STATE_STOPPED) gState = MRT_STATE_FINISHED;
            --gActive;
        }
        gIdle.notify_all();
        gState = MRT_STATE_IDLE;
    };
    try {
        std::thread(body).detach();
    } catch (const std::exception&) {  // std::system_error: no thread was started
        // undo what the thread would have undone, so later initialize / reset / wait calls do not
        // block on it, and hand the pixels back (the JNI caller unlocks its bitmap in done)
        {
            std::lock_guard<std::mutex> lock(gMutex);
            --gActive;
        }
        gIdle.notify_all();
        if (done != nullptr) done(user);
        gFinished = true;
        gRendered.notify_all();
        gState = MRT_STATE_IDLE;
    }
}

void mrt_android_render_into_bitmap(int32_t* pixels, int32_t nThreads) {
    mrt_android_render_into_bitmap_cb(pixels, nThreads, nullptr, nullptr);
}

void mrt_android_wait_render(void) {
    std::unique_lock<std::mutex> lock(gMutex);
    gIdle.wait(lock, [] { return gActive == 0; });
}

void mrt_android_start_render(int32_t wait) {  // :406-426
    if (wait != 0) {
        std::unique_lock<std::mutex> lock(gMutex);
        gRendered.wait(lock, [] { return gFinished.load(); });
        gFinished = false;
    }
    gState = MRT_STATE_BUSY;
}

void mrt_android_stop_render(int32_t wait) {  // :428-462
    gState = MRT_STATE_STOPPED;
    std::unique_lock<std::mutex> lock(gMutex);
    if (gRenderer != nullptr) mrt_stop_render(gRenderer.get());
    if (wait != 0) {
        while (!gFinished) {
            if (gRenderer != nullptr) {
                mrt_stop_render(gRenderer.get());
                break;
            }
            gRendered.wait_for(lock, std::chrono::seconds(3), [] { return gFinished.load(); });
        }
    }
}

void mrt_android_finish_render(void) {  // :718-741
    std::lock_guard<std::mutex> lock(gMutex);
    gState = MRT_STATE_FINISHED;
    if (gRenderer != nullptr) mrt_stop_render(gRenderer.get());
    gState = MRT_STATE_IDLE;
    gFps = 0.0F;
    gTimeRenderer = 0;
    gFinished = true;
}

int32_t mrt_android_state(void) { return gState.load(); }
float mrt_android_fps(void) { return gFps.load(); }
int64_t mrt_android_time_renderer(void) { return gTimeRenderer.load(); }
int32_t mrt_android_number_of_lights(void) { return gNumLights.load(); }

int32_t mrt_android_sample(void) {
    const std::shared_ptr<mrt_renderer> r = current();
    return r != nullptr ? mrt_get_sample(r.get()) : 0;
}

int32_t mrt_android_resize(int32_t size) {  // roundDownToMultipleOf(size, sqrt(NumberOfTiles) = 16)
    const int32_t rest = size % 16;
    return rest > 1 ? size - rest : size;
}

int64_t mrt_android_vertices(float* out) {
    const std::shared_ptr<mrt_renderer> r = current();
    if (r == nullptr) return 0;
    const int64_t n = mrt_preview_arrays(r.get(), out, nullptr, nullptr);
    return n < 0 ? 0 : 12 * n;
}

int64_t mrt_android_colors(float* out) {
    const std::shared_ptr<mrt_renderer> r = current();
    if (r == nullptr) return 0;
    const int64_t n = mrt_preview_arrays(r.get(), nullptr, out, nullptr);
    return n < 0 ? 0 : 12 * n;
}

int64_t mrt_android_camera(float* out) {
    const std::shared_ptr<mrt_renderer> r = current();
    if (r == nullptr) return 0;
    return mrt_preview_arrays(r.get(), nullptr, nullptr, out) < 0 ? 0 : 20;
}

void mrt_android_reset(void) {
    std::unique_lock<std::mutex> lock(gMutex);
    stopAndWait(lock);
    gRenderer.reset();
    gObj.clear();
    gMtl.clear();
    gCam.clear();
    gTextures.clear();
    gState = MRT_STATE_IDLE;
    gFinished = true;
    gFps = 0.0F;
    gTimeRenderer = 0;
    gNumLights = 0;
}

}  // extern "C"
