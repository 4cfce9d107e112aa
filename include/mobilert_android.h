/*
 * mobilert_android.h - the Android front end's native session over the MI355X render path.
 *
 * The reference's JNI layer (app/System_dependent/Android_JNI/JNI_layer.cpp) keeps one renderer
 * and a small state machine in file statics and exports them as Java_puscas_mobilertapp_* methods.
 * This header is that session with plain C types: the JNI exports themselves
 * (mobileraytracer_amd/jni/mrt_jni.cpp, built with the Android NDK) only unpack the Java objects
 * and call these functions, one each:
 *
 *   mrt_android_read_file          MainActivity.readFile          (JNI_layer.cpp:994-1063)
 *   mrt_android_initialize         MainRenderer.rtInitialize      (:464-716)
 *   mrt_android_render_into_bitmap MainRenderer.rtRenderIntoBitmap (:743-901)
 *   mrt_android_finish_render      MainRenderer.rtFinishRender    (:718-741)
 *   mrt_android_start_render       DrawView.rtStartRender         (:406-426)
 *   mrt_android_stop_render        DrawView.rtStopRender          (:428-462)
 *   mrt_android_number_of_lights   DrawView.rtGetNumberOfLights   (:1065-1074)
 *   mrt_android_state / fps / time_renderer / sample
 *                                  RenderTask.rtGetState / rtGetFps / rtGetTimeRenderer / rtGetSample (:903-963)
 *   mrt_android_resize             MainActivity.rtResize          (:965-981)
 *   mrt_android_vertices / colors / camera
 *                                  MainRenderer.rtInitVerticesArray / rtInitColorsArray /
 *                                  rtInitCameraArray (:153-389; the JNI side wraps the floats in a
 *                                  DirectByteBuffer that rtFreeNativeBuffer, :1076-1090, releases)
 */
#ifndef MOBILERT_ANDROID_H
#define MOBILERT_ANDROID_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* JNI_layer.hpp:12-13 */
enum mrt_android_state { MRT_STATE_IDLE = 0, MRT_STATE_BUSY = 1, MRT_STATE_FINISHED = 2, MRT_STATE_STOPPED = 3 };

/* What rtInitialize reads from the Java Config object (getScene, getShader, getAccelerator,
 * getConfigResolution().getWidth/getHeight, getConfigSamples().getSamplesPixel/getSamplesLight,
 * getObjFilePath). */
typedef struct mrt_android_config {
    int32_t scene;
    int32_t shader;
    int32_t accelerator;
    int32_t width;
    int32_t height;
    int32_t samplesPixel;
    int32_t samplesLight;
    const char *objFilePath;
} mrt_android_config;

/* readFile: the bytes of one file picked by the user.  ".obj", ".mtl", ".cam" are kept as the scene
 * definition for the next initialize; anything else is a texture, cached by its file name. */
void mrt_android_read_file(const char *path, const uint8_t *bytes, int64_t size);
/* rtInitialize: cancels a render still running and waits for its thread, then builds the renderer (built-in scenes 0-3, else the OBJ read before, whose
 * definitions are then dropped).  Returns triangles + spheres + planes, or -1 (out of memory or
 * the OBJ could not be processed), -2 (any other error; message in mrt_last_error), -3. */
int32_t mrt_android_initialize(const mrt_android_config *config);
/* rtRenderIntoBitmap: renders frames into pixels (width x height ABGR int32, kept by the caller
 * until the state leaves BUSY) on a detached thread while the state is BUSY (one frame), updating
 * fps / sample, then FINISHED unless stopped, then IDLE.  nThreads is the reference's and unused. */
void mrt_android_render_into_bitmap(int32_t *pixels, int32_t nThreads);
/* The same, and done(user) is called on the render thread once its last frame has returned, i.e.
 * once nothing writes pixels any more (the JNI layer unlocks the Android bitmap there, as the
 * reference's render thread does, JNI_layer.cpp:850-854). */
typedef void (*mrt_android_done_fn)(void *user);
void mrt_android_render_into_bitmap_cb(int32_t *pixels, int32_t nThreads, mrt_android_done_fn done, void *user);
/* Blocks until no render thread is running (every pixels buffer handed over is released). */
void mrt_android_wait_render(void);
/* rtStartRender: with wait, blocks until the previous render finished; state BUSY. */
void mrt_android_start_render(int32_t wait);
/* rtStopRender: state STOPPED, the renderer's cooperative cancel. */
void mrt_android_stop_render(int32_t wait);
/* rtFinishRender: cancels, state IDLE, fps and time 0. */
void mrt_android_finish_render(void);
int32_t mrt_android_state(void);
float mrt_android_fps(void);
int64_t mrt_android_time_renderer(void);   /* milliseconds the shader / accelerator build took */
int32_t mrt_android_sample(void);
int32_t mrt_android_number_of_lights(void);
/* rtResize: roundDownToMultipleOf(size, 16) (Utils.cpp:26-31: rest > 1 ? size - rest : size) */
int32_t mrt_android_resize(int32_t size);
/* the GL preview arrays (mrt_preview_arrays of the current renderer): float counts returned
 * (12 per triangle; 20 for the camera), 0 without a renderer; NULL out only counts */
int64_t mrt_android_vertices(float *out);
int64_t mrt_android_colors(float *out);
int64_t mrt_android_camera(float *out);
/* drops the renderer (after cancelling and waiting for a running render) and every cached file
 * (JNI_OnUnload) */
void mrt_android_reset(void);

#ifdef __cplusplus
}
#endif

#endif
