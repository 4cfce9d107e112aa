// mrt_jni.cpp - the Android front end's JNI exports over the MI355X render path.
//
// Same exported names and Java-visible behaviour as the reference's
// app/System_dependent/Android_JNI/JNI_layer.cpp (file:line below), so MainRenderer.java,
// DrawView.java, RenderTask.kt and MainActivity.java call it unchanged.  Each export only
// unpacks Java objects and forwards to the native session of include/mobilert_android.h
// (mobileraytracer_amd/csrc/mrt_android.cpp), which holds the renderer and the state machine and
// is exercised by tests/test_android_session.py.
//
// Built with the Android NDK (jni.h, android/bitmap.h, -ljnigraphics) into the app's native
// library together with libmobilert_amd; this image has no NDK, so build() does not compile it.
// Exceptions become Java exceptions as the reference's handleException does (:114-126):
// LowMemoryException for std::bad_alloc, RuntimeException otherwise.
#include <android/bitmap.h>
#include <jni.h>

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <unistd.h>
#include <vector>

#include "mobilert_amd.h"
#include "mobilert_android.h"

namespace {

JavaVM* javaVM_ = nullptr;

void throwJava(JNIEnv* env, const char* clazz, const char* message) {
    const jclass c = env->FindClass(clazz);
    if (c != nullptr) env->ThrowNew(c, message);
}

template <class F>
auto guarded(JNIEnv* env, F&& f, decltype(f()) onError) -> decltype(f()) {
    try {
        return f();
    } catch (const std::bad_alloc& e) {
        throwJava(env, "puscas/mobilertapp/exceptions/LowMemoryException", e.what());
    } catch (const std::exception& e) {
        throwJava(env, "java/lang/RuntimeException", e.what());
    } catch (...) {
        throwJava(env, "java/lang/RuntimeException", "unknown native error");
    }
    return onError;
}

jint callInt(JNIEnv* env, jobject obj, const char* method) {
    const jclass c = env->GetObjectClass(obj);
    return env->CallIntMethod(obj, env->GetMethodID(c, method, "()I"));
}

jobject callObject(JNIEnv* env, jobject obj, const char* method, const char* signature) {
    const jclass c = env->GetObjectClass(obj);
    return env->CallObjectMethod(obj, env->GetMethodID(c, method, signature));
}

// a float array in native memory handed to Java as a DirectByteBuffer; Java releases it through
// rtFreeNativeBuffer (:1076-1090)
jobject directFloats(JNIEnv* env, int64_t (*fill)(float*)) {
    const int64_t n = fill(nullptr);
    if (n <= 0) return nullptr;
    float* buf = new float[static_cast<size_t>(n)];
    fill(buf);
    const jobject direct = env->NewDirectByteBuffer(buf, n * static_cast<jlong>(sizeof(jfloat)));
    if (direct == nullptr) {
        delete[] buf;
        throw std::runtime_error("JNIEnv::NewDirectByteBuffer failed to allocate native memory!");
    }
    return direct;
}

// The locked Android bitmap, released by the session's render thread once its last frame has
// returned (mrt_android_render_into_bitmap_cb's callback): it attaches to the VM, unlocks the pixels
// and drops the global reference, as the reference's render thread does after renderFrame
// (JNI_layer.cpp:850-869).  Nothing writes the pixels after that point.
void unlockBitmap(void* user) {
    const jobject bitmap = static_cast<jobject>(user);
    JNIEnv* tenv = nullptr;
    if (javaVM_ != nullptr && javaVM_->AttachCurrentThread(&tenv, nullptr) == JNI_OK) {
        AndroidBitmap_unlockPixels(tenv, bitmap);
        tenv->DeleteGlobalRef(bitmap);
        javaVM_->DetachCurrentThread();
    }
}

}  // namespace

extern "C" {

JNIEXPORT jint JNICALL JNI_OnLoad(JavaVM* jvm, void* /*reserved*/) {  // :128-146
    errno = 0;
    javaVM_ = jvm;
    return JNI_VERSION_1_6;
}

JNIEXPORT void JNICALL JNI_OnUnload(JavaVM* /*jvm*/, void* /*reserved*/) {  // :148-151
    mrt_android_reset();
    javaVM_ = nullptr;
}

JNIEXPORT jobject JNICALL Java_puscas_mobilertapp_MainRenderer_rtInitCameraArray(JNIEnv* env, jobject /*thiz*/) {
    return guarded(env, [&] { return directFloats(env, mrt_android_camera); }, static_cast<jobject>(nullptr));
}

JNIEXPORT jobject JNICALL Java_puscas_mobilertapp_MainRenderer_rtInitVerticesArray(JNIEnv* env, jobject /*thiz*/) {
    return guarded(env, [&] { return directFloats(env, mrt_android_vertices); }, static_cast<jobject>(nullptr));
}

JNIEXPORT jobject JNICALL Java_puscas_mobilertapp_MainRenderer_rtInitColorsArray(JNIEnv* env, jobject /*thiz*/) {
    return guarded(env, [&] { return directFloats(env, mrt_android_colors); }, static_cast<jobject>(nullptr));
}

JNIEXPORT jobject JNICALL Java_puscas_mobilertapp_MainRenderer_rtFreeNativeBuffer(JNIEnv* env, jobject /*thiz*/,
                                                                                jobject bufferRef) {
    if (bufferRef != nullptr) delete[] static_cast<float*>(env->GetDirectBufferAddress(bufferRef));
    return nullptr;
}

JNIEXPORT void JNICALL Java_puscas_mobilertapp_DrawView_rtStartRender(JNIEnv* env, jobject /*thiz*/, jboolean wait) {
    mrt_android_start_render(wait ? 1 : 0);
    env->ExceptionClear();
}

JNIEXPORT void JNICALL Java_puscas_mobilertapp_DrawView_rtStopRender(JNIEnv* env, jobject /*thiz*/, jboolean wait) {
    mrt_android_stop_render(wait ? 1 : 0);
    env->ExceptionClear();
}

// :464-716: the Java Config object's getters, then the native session
JNIEXPORT jint JNICALL Java_puscas_mobilertapp_MainRenderer_rtInitialize(JNIEnv* env, jobject /*thiz*/,
                                                                         jobject localConfig) {
    const jobject resolution =
        callObject(env, localConfig, "getConfigResolution", "()Lpuscas/mobilertapp/configs/ConfigResolution;");
    const jobject samples = callObject(env, localConfig, "getConfigSamples", "()Lpuscas/mobilertapp/configs/ConfigSamples;");
    const auto objPath = static_cast<jstring>(callObject(env, localConfig, "getObjFilePath", "()Ljava/lang/String;"));
    const char* objChars = objPath != nullptr ? env->GetStringUTFChars(objPath, nullptr) : nullptr;
    const std::string obj = objChars != nullptr ? objChars : "";
    if (objChars != nullptr) env->ReleaseStringUTFChars(objPath, objChars);
    mrt_android_config c{};
    c.scene = callInt(env, localConfig, "getScene");
    c.shader = callInt(env, localConfig, "getShader");
    c.accelerator = callInt(env, localConfig, "getAccelerator");
    c.width = callInt(env, resolution, "getWidth");
    c.height = callInt(env, resolution, "getHeight");
    c.samplesPixel = callInt(env, samples, "getSamplesPixel");
    c.samplesLight = callInt(env, samples, "getSamplesLight");
    c.objFilePath = obj.c_str();
    const jint res = mrt_android_initialize(&c);
    if (res == -1) throwJava(env, "puscas/mobilertapp/exceptions/LowMemoryException", mrt_last_error());
    if (res == -2 || res == -3) throwJava(env, "java/lang/RuntimeException", mrt_last_error());
    return res;
}

JNIEXPORT void JNICALL Java_puscas_mobilertapp_MainRenderer_rtFinishRender(JNIEnv* env, jobject /*thiz*/) {
    mrt_android_finish_render();
    env->ExceptionClear();
}

// :743-901: the bitmap stays locked while the session's render thread writes it; the render
// thread unlocks it (unlockBitmap) once its last frame has returned
JNIEXPORT void JNICALL Java_puscas_mobilertapp_MainRenderer_rtRenderIntoBitmap(JNIEnv* env, jobject /*thiz*/,
                                                                               jobject localBitmap, jint nThreads) {
    guarded(env, [&] {
        const jobject bitmap = env->NewGlobalRef(localBitmap);
        void* pixels = nullptr;
        if (AndroidBitmap_lockPixels(env, bitmap, &pixels) != ANDROID_BITMAP_RESULT_SUCCESS) {
            env->DeleteGlobalRef(bitmap);
            throw std::runtime_error("Couldn't lock the Android bitmap pixels.");
        }
        mrt_android_render_into_bitmap_cb(static_cast<int32_t*>(pixels), nThreads, unlockBitmap, bitmap);
        return 0;
    }, 0);
}

JNIEXPORT jint JNICALL Java_puscas_mobilertapp_RenderTask_rtGetState(JNIEnv* env, jobject /*thiz*/) {
    env->ExceptionClear();
    return mrt_android_state();
}

JNIEXPORT jfloat JNICALL Java_puscas_mobilertapp_RenderTask_rtGetFps(JNIEnv* env, jobject /*thiz*/) {
    if (errno == ETIMEDOUT || errno == EBADF) errno = 0;  // :921-925
    env->ExceptionClear();
    return mrt_android_fps();
}

JNIEXPORT jlong JNICALL Java_puscas_mobilertapp_RenderTask_rtGetTimeRenderer(JNIEnv* env, jobject /*thiz*/) {
    env->ExceptionClear();
    return mrt_android_time_renderer();
}

JNIEXPORT jint JNICALL Java_puscas_mobilertapp_RenderTask_rtGetSample(JNIEnv* env, jobject /*thiz*/) {
    if (errno == EBADF) errno = 0;  // :948-951
    env->ExceptionClear();
    return mrt_android_sample();
}

JNIEXPORT jint JNICALL Java_puscas_mobilertapp_MainActivity_rtResize(JNIEnv* env, jobject /*thiz*/, jint size) {
    env->ExceptionClear();
    return mrt_android_resize(size);
}

JNIEXPORT void JNICALL Java_puscas_mobilertapp_MainActivity_resetErrno(JNIEnv* env, jclass /*clazz*/) {
    errno = 0;
    env->ExceptionClear();
}

// :994-1063: the file behind a descriptor the Java side opened (scene definition or texture)
JNIEXPORT void JNICALL Java_puscas_mobilertapp_MainActivity_readFile(JNIEnv* env, jobject /*thiz*/, jint fileDescriptor,
                                                                     jlong fileSize, jstring jFilePath) {
    if (errno == EACCES || errno == ENOTSOCK || errno == EPERM || errno == ENOENT) errno = 0;
    const char* chars = env->GetStringUTFChars(jFilePath, nullptr);
    const std::string path = chars != nullptr ? chars : "";
    if (chars != nullptr) env->ReleaseStringUTFChars(jFilePath, chars);
    std::vector<uint8_t> bytes(static_cast<size_t>(fileSize > 0 ? fileSize : 0));
    size_t got = 0;
    while (got < bytes.size()) {
        const ssize_t n = ::read(fileDescriptor, bytes.data() + got, bytes.size() - got);
        if (n <= 0) break;
        got += static_cast<size_t>(n);
    }
    mrt_android_read_file(path.c_str(), bytes.data(), static_cast<int64_t>(got));
}

JNIEXPORT jint JNICALL Java_puscas_mobilertapp_DrawView_rtGetNumberOfLights(JNIEnv* env, jobject /*thiz*/) {
    env->ExceptionClear();
    return mrt_android_number_of_lights();
}

}  // extern "C"
