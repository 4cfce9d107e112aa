/*
 * mobilert_amd.h - C-ABI of the MI355X (gfx950) render hot path of MobileRT.
 *
 * Plain C: opaque handles, plain pointers and sizes, int status codes (0 = ok, < 0 = error,
 * message from mrt_last_error()).  Every entry point names the reference interface it
 * replaces (paths relative to TiagoMSSantos/MobileRayTracer):
 *
 *   mrt_create                Shader ctor + Renderer ctor as assembled by work_thread
 *                             (app/System_dependent/Native/C_wrapper.cpp:36-211) and by
 *                             JNI rtInitialize (app/System_dependent/Android_JNI/JNI_layer.cpp:464-716)
 *   mrt_render_frame          Renderer::renderFrame(int32_t *bitmap, int32_t numThreads)
 *                             (app/MobileRT/Renderer.hpp:57, Renderer.cpp:53-88)
 *   mrt_render_frame_device   the same, bitmap resident in device memory (no PCIe in the window)
 *   mrt_stop_render           Renderer::stopRender (Renderer.cpp:93-99); JNI rtStopRender
 *   mrt_get_sample            Renderer::getSample (Renderer.cpp:177-179); JNI rtGetSample
 *   mrt_get_total_casted_rays Renderer::getTotalCastedRays (Renderer.cpp:204-207)
 *   mrt_get_scene_info        Shader::getTriangles/getLights/getPlanes/getSpheres/getMaterials
 *                             sizes (Shader.hpp:92-100); C_wrapper.cpp:199-202 log lines
 *   mrt_primary_hits          first closest hit of every camera ray (config C2 parity dump)
 *   mrt_destroy               renderer_.reset() (C_wrapper.cpp:265)
 *
 * The desktop symbols RayTrace(Config&, bool) / stopRender() of
 * app/System_dependent/Native/C_wrapper.h:12-20 are declared in mobilert_amd.hpp (they take
 * a C++ reference) and exported by the same library.
 */
#ifndef MOBILERT_AMD_H
#define MOBILERT_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mrt_renderer mrt_renderer;

/* Mirrors MobileRT::Config (app/MobileRT/Config.hpp:12-83) field for field, minus the
 * bitmap vector, plus the GPU-only knobs at the end. */
typedef struct mrt_config {
    int32_t width;
    int32_t height;
    int32_t threads;      /* kept for API parity; the GPU path does not use it */
    int32_t shader;       /* 1 Whitted, 2 PathTracer (C_wrapper.cpp:154-193) */
    int32_t sceneIndex;   /* 0 built-in Cornell box, < 0 or > 3 OBJ (C_wrapper.cpp:76-140) */
    int32_t samplesPixel;
    int32_t samplesLight;
    int32_t repeats;
    int32_t accelerator;  /* Shader.hpp:20-24: 1 Naive, 2 RegularGrid, 3 BVH; any other value
                             builds no accelerator (only lights are hit) */
    int32_t printStdOut;
    const char *objFilePath;
    const char *mtlFilePath;
    const char *camFilePath;
    /* GPU-only */
    int32_t maxDepth;     /* RayDepthMax (Constants.hpp:45); <= 0 -> 6 */
    int32_t rankIndex;    /* screen-tile shard owned by this process */
    int32_t rankCount;    /* number of shards (GPUs); <= 0 -> 1 */
    int32_t device;       /* HIP device ordinal, -1 = current device */
    int32_t cull;         /* near-first traversal with t-culling of the triangle BVH:
                           * 0 none (the reference's visit set; exact), 1 fast: a box whose entry
                           * exceeds best * (1 + 2^-10) is skipped (NOT exact for every input:
                           * a grazing Moller-Trumbore hit can lie before its box), 2 certified:
                           * every box skipped only on a rigorous bound of Moller-Trumbore's
                           * rounding (exact, slow), 3 exact (recommended; RayTrace, the Android
                           * session and the Python Config use it): inner boxes never skipped,
                           * leaves skipped on the certified bound of their own triangles.  See
                           * DESIGN.md section 3. */
    int32_t maxPathsPerPass; /* <= 0 -> automatic chunk size */
    int32_t progressive;  /* 1: one pass per sample; bitmap and mrt_get_sample() updated after
                           * each (Renderer.cpp:53-88).  0: all samples in flight at once.
                           * The final bitmap is the same. */
    /* A device group (Renderer::renderFrame spreading one frame over its workers,
     * Renderer.cpp:62-82, with the workers on GPUs): deviceCount > 1 renders every frame as
     * deviceCount screen-tile shards, shard i on HIP device devices[i] from a host thread of its
     * own, assembled on devices[0] (peer copies over xGMI, then one unpack launch), which holds
     * the device bitmap of mrt_render_frame_device.  A repeated ordinal puts several shards on
     * one GPU.  The bitmap and the ray counts equal the single-GPU frame's.  `device`, rankIndex
     * and rankCount must be left at their defaults (-1 / 0 / <= 1).  deviceCount <= 1: one GPU. */
    const int32_t *devices;
    int32_t deviceCount;
} mrt_config;

typedef struct mrt_scene_info {
    int64_t triangles;
    int64_t lights;
    int64_t planes;
    int64_t spheres;
    int64_t materials;
    int64_t triangleNodes;
    int64_t triangleBvhDepth;
    int64_t pixelSlots;      /* pixels rendered by this shard per sample */
    int64_t pixelSlotsMax;   /* max over shards (size of a gather slot) */
    int64_t deviceBytes;     /* device memory held by the renderer */
    int64_t shadowStreamConcurrent; /* 1: the shadow walks run on their own stream beside the render
                                       chain (checked at mrt_create: the two streams' kernels overlap
                                       in time, i.e. they feed different hardware queues, whatever
                                       streams the process created before); 0: serialised */
    int64_t shadowStreamsTried;     /* shadow streams created until one ran concurrently */
    int64_t deviceCount;            /* GPUs of the renderer's device group (1: a single GPU) */
} mrt_scene_info;

typedef struct mrt_frame_stats {
    uint64_t rays;          /* camera + diffuse + specular + transmission rays */
    uint64_t shadowRays;
    uint64_t primaryRays;
    uint64_t nodeRecords;   /* counting pass only: BVH child records fetched by closest-hit rays */
    uint64_t triTests;      /* counting pass only: ray/triangle tests of closest-hit rays */
    uint64_t shadowNodeRecords; /* counting pass only: the same for shadow (any-hit) rays */
    uint64_t shadowTriTests;
    double traceMs;         /* profiling: summed duration of closest-hit trace launches */
    double shadowMs;        /* profiling: summed duration of any-hit trace launches */
    double frameMs;         /* whole frame on the render stream, host wall time; a device group: the
                               group's wall time (the per-kernel ms fields and launch counts are
                               summed over its shards) */
    int64_t traceLaunches;
    int64_t shadowLaunches;
    double shadeMs;         /* profiling: summed duration of the shading launches */
    uint64_t levelRays[16];       /* rays of depth 1..16 (1 = camera rays) */
    uint64_t levelShadowRays[16]; /* shadow rays built at depth 1..16 */
    double levelTraceMs[16];      /* profiling: closest-hit trace time per depth */
    double levelShadowMs[16];     /* profiling: any-hit trace time per depth */
    uint64_t maxNodeRecordsPerRay; /* counting pass only: most node records one ray fetched */
    uint64_t walkedRays;           /* closest-hit rays traversed: `rays` minus the depth-capped last
                                      level's, whose walk is skipped (tuning key 7) */
    uint64_t shadedVertices;       /* counting pass only: hits k_shade shaded (not emissive, under the
                                      depth cap) */
    int64_t shadeLaunches;         /* k_shade launches of the frame */
    uint64_t leafRecords;          /* counting pass only: walk-tree leaf records (exact leaf boxes)
                                      fetched by closest-hit rays */
    uint64_t shadowLeafRecords;    /* ... and by shadow rays */
    uint64_t levelNodeRecords[16]; /* counting pass only: nodeRecords of the closest-hit rays of depth 1..16 */
    uint64_t levelTriTests[16];    /* ... triTests */
    uint64_t levelLeafRecords[16]; /* ... leafRecords */
    double fusedMs;                /* profiling: summed duration of the fused level-1 launches
                                      (k_trace_packet_shade: camera rays generated, walked and shaded;
                                      not in traceMs / shadeMs) */
    int64_t fusedLaunches;         /* fused level-1 launches of the frame (counted in shadeLaunches too) */
    uint64_t levelShadedVertices[16]; /* counting pass only: shadedVertices of depth 1..16 */
    uint64_t shadowOccluded;       /* counting pass only: occluded shadow rays */
    uint64_t walkPhases[16];       /* counting pass only, the persistent walks (closest hit, then any hit):
                                      wave iterations and the lanes active in them of the inner-node phase,
                                      the leaf phase and the triangle loop: {iters, lanes} x 3 x 2; then per
                                      walk, summed over inner iterations, the wave's lanes without a ray
                                      and with a finished one: {idle, done} x 2 */
    uint64_t packetWaveRecords[3]; /* counting pass only, the level-1 packet walk (scalar loads, each record
                                      fetched once for the wave's 64 rays): per wave, inner nodes visited
                                      (128 B each), leaf records loaded (48 B), triangle records loaded (48 B) */
} mrt_frame_stats;

/* A named byte buffer (a map_Kd texture file handed over by the Android front end). */
typedef struct mrt_blob {
    const char *name;     /* file name (the part after the last '/') */
    const uint8_t *bytes;
    int64_t size;
} mrt_blob;

const char *mrt_last_error(void);
/* digest of the sources the library was built from (Makefile: sha256 of the csrc sources and
 * headers, first 16 hex digits, then any extra compile flags) */
const char *mrt_build_stamp(void);
int mrt_create(const mrt_config *cfg, mrt_renderer **out);
/* mrt_create with the OBJ / MTL / CAM given as text and the textures as named blobs, as the
 * Android front end hands them over (MainActivity.readFile -> JNI readFile, JNI_layer.cpp:994-1063,
 * then rtInitialize, :464-716, which parses them from memory).  cfg's file paths are ignored for
 * OBJ scenes (sceneIndex outside 0-3); an empty obj fails with "OBJ file not read!" (:552-555).
 * Such a renderer keeps a host copy of its triangles for mrt_preview_arrays. */
int mrt_create_from_memory(const mrt_config *cfg, const char *obj, int64_t objLen, const char *mtl, int64_t mtlLen,
                           const char *cam, int64_t camLen, const mrt_blob *textures, int32_t nTextures,
                           mrt_renderer **out);
/* The GL preview arrays of the Android front end (rtInitVerticesArray / rtInitColorsArray /
 * rtInitCameraArray, JNI_layer.cpp:153-389), for a renderer made by mrt_create_from_memory:
 * vertices[12 T] (A, B, C of every triangle in BVH order, xyz with z negated, w 1), colors[12 T]
 * (per triangle: Kd, or Ks / Kt / Le where greater in all components, w 1, three times), camera[20]
 * (position, direction, up, right as xyz1; then hFov, vFov in degrees, 0, 0 for a perspective
 * camera or 0, 0, sizeH / 2, sizeV / 2 for an orthographic one).  NULL outputs are skipped.
 * Returns T (triangles) or -1. */
int64_t mrt_preview_arrays(const mrt_renderer *r, float *vertices, float *colors, float *camera);
void mrt_destroy(mrt_renderer *r);
/* bitmap: host array of width*height int32 ABGR pixels, updated in place */
int mrt_render_frame(mrt_renderer *r, int32_t *bitmap);
/* d_bitmap: device array (width*height) or NULL; d_packed: device array of pixelSlots
 * entries (this shard's pixels in slot order) or NULL; stream: hipStream_t or NULL */
int mrt_render_frame_device(mrt_renderer *r, int32_t *d_bitmap, int32_t *d_packed, void *stream);
/* rank 0 frame assembly: d_gathered holds rankCount slices of pixelSlotsMax entries */
int mrt_unpack_gathered(mrt_renderer *r, const int32_t *d_gathered, int32_t *d_bitmap, void *stream);
int mrt_stop_render(mrt_renderer *r);
int32_t mrt_get_sample(const mrt_renderer *r);
uint64_t mrt_get_total_casted_rays(const mrt_renderer *r);
int mrt_get_scene_info(const mrt_renderer *r, mrt_scene_info *info);
/* enable per-launch HIP event timing (1) and/or node/triangle counting (2) */
int mrt_set_profiling(mrt_renderer *r, int32_t flags);
int mrt_get_frame_stats(const mrt_renderer *r, mrt_frame_stats *stats);
/* counting mode: the last frame's wave log, out[2][16][8192][4] (closest / any-hit walk x level x
 * wave: start, end in 100 MHz ticks, rays fetched, child records fetched; zero where no wave
 * ran).  Returns the entry count (1,048,576) or -1; out NULL only counts. */
int64_t mrt_wave_log(mrt_renderer *r, uint64_t *out);
/* The in-process plugin surface of app/MobileRT/Renderer.hpp:41-63 (include/mobilert_renderer.hpp
 * builds on these).  mrt_set_camera replaces the renderer's camera: kind 0 Perspective(position,
 * lookAt, up, hFov, vFov in degrees; Perspective.cpp:8-14, Camera.cpp:14-19), 1 Orthographic(position,
 * lookAt, up, sizeH, sizeV; Orthographic.cpp:7-13).  mrt_set_pixel_sampler: the Renderer's
 * samplerPixel_, kind 0 Constant(value) (Constant.cpp:9-11), 1 StaticHaltonSeq (the deterministic
 * table draws), -1 (default) as C_wrapper.cpp:144-148: StaticHaltonSeq iff samplesPixel > 1.
 * mrt_set_max_point: DepthMap's maxPoint (DepthMap.cpp; C_wrapper.cpp:79-131 passes maxDist).
 * Each applies from the next frame; 0 on success. */
int mrt_set_camera(mrt_renderer *r, int32_t kind, const float *position, const float *lookAt, const float *up,
                   float a, float b);
int mrt_set_pixel_sampler(mrt_renderer *r, int32_t kind, float value);
int mrt_set_max_point(mrt_renderer *r, const float *maxPoint);
/* tuning knobs for A/B measurement (results are identical for every value):
 * key 1 = trace walk: 0 per-wave 64-ray batches with the plain DFS of BVH.hpp:327-384,
 *         1 persistent while-while walk (default),
 * key 2 = cull mode of walk 1: 0 none, 1 fast (inexact), 2 certified, 3 exact (mrt_config.cull),
 * key 3 = shadow rays on the same stream (0) or their own stream (1, default),
 * key 5 = shadow walk child order: 0 near first, 1 far first (default),
 * key 6 = shadow walk grid, percent of its occupancy grid (1-100; 0 default: 50-75 by paths per walk lane),
 * key 7 = skip the closest-hit walk of the depth-capped last level (1, default),
 * key 8 = tail donation: idle lanes of a level's tail walk subtrees of their wave's rays (0, 1 default),
 * key 9 = idle lanes before a walk wave fetches new rays (1-64, default 32),
 * key 10 = k_shade's lean instantiation where it applies (1, default) or always the general one (0),
 * key 11 = k_shade workgroups per CU (-1 default: 14; 0: 8; 1-64: that many),
 * key 16 = camera rays by the wave-coherent packet walk in cull modes 0 and 3 (1, default) or the
 *          per-lane walk (0); refused (-1) when the walk tree needs a deeper traversal stack than
 *          the packet walk's LDS stack (kPacketStack),
 * key 17 = level 1 fused: camera rays generated, packet-walked and shaded in one launch (1, where it
 *          applies: BVH, packet walk, Whitted / PathTracer, untextured, lean shading, no counting) or
 *          the separate raygen / walk / shade launches (0); -1 (default since round 6): fused below
 *          12 paths per resident walk lane (a shard of C4 at N >= 2), separate above (DESIGN.md
 *          section 7),
 * key 27 = the last shadow walk of a pass on the render stream with the closest-hit spill stacks
 *          (1, default) or on the shadow stream (0),
 * key 28 = at most this many workgroups per walk launch (0, default: the occupancy grid; 1-65536):
 *          a test knob, every grid size walks every ray,
 * key 33 = where level 1 is not fused (key 17), the packet walk generates the camera rays itself and
 *          stores the records the shading reads (1), or k_shade regenerates them too (2, Whitted /
 *          PathTracer; default), or the walk reads those of a k_raygen launch (0),
 * key 34 = level 1's resolve folded into the per-pixel accumulation, one launch (1, default), or the
 *          resolve and k_accumulate launched separately (0),
 * key 35 = the shading of level L waits for the shadow walk of level L - 2 (1: round 1's order, when
 *          shadow queues alternated by level parity) or not (0, default).
 * (Keys 4, 12-15, 18, 19-25, 29, 30, 32, 36 - binned emission, queue sorting, graph replay, the tile
 * kernel, a shadow-occluder probe, the deeper levels' walk and shading in one launch, a CU-masked
 * shadow stream, k_shade's vertices binned by shading class, the shadow walks yielding to the next
 * level's shading, a level's closest-hit and shadow walks in one launch - measured slower and were
 * removed.) */
int mrt_set_tuning(mrt_renderer *r, int32_t key, int32_t value);
int mrt_get_tuning(const mrt_renderer *r, int32_t key, int32_t *value);
/* per pixel (width*height host arrays): kind 0 miss / 1 plane / 2 sphere / 3 triangle /
 * 4 light; index in the scene's input order (-1 on miss); t = hit distance */
int mrt_primary_hits(mrt_renderer *r, int32_t *kind, int32_t *index, float *t);
/* Host only (no GPU): the scene's triangle BVH as built for the device (BVH.hpp:161-283,
 * built in parallel with the serial build's result).  Returns the node-array length N
 * (slots; unreachable slots are zero) or -1.  With non-NULL outputs fills boxes[N*6]
 * (min xyz, max xyz), offsets[N] / counts[N] (BVHNode::indexOffset / numPrimitives) and
 * order[triangles] (input index of each triangle in BVH order). */
int64_t mrt_triangle_bvh(const mrt_config *cfg, float *boxes, int32_t *offsets, int32_t *counts, int32_t *order);
/* Host only: the quantized wide walk tree the BVH walk traverses:
 * returns the node count or -1; with non-NULL outputs fills nodes (count x 4W uint32: 3W box
 * words, child c's axis a at 3c + a as min | max << 16; W child references; W = the walk width,
 * root[2]), grid[6] (origin xyz, step xyz) and
 * root[3] (reference, triangles, W). */
int64_t mrt_walk_tree(const mrt_config *cfg, uint32_t *nodes, float *grid, int32_t *root);
/* Host only: the RegularGrid accelerator's build (RegularGrid.hpp:112-289, gridSize 32) for one
 * primitive kind of the scene cfg names (kind 0 planes, 1 spheres, 2 triangles).  Returns the
 * total list length L or -1; with non-NULL outputs fills world[12] (min xyz, max xyz, cellSize
 * xyz, cellSizeInverted xyz), start[32768 + 1] (cell c's list is items[start[c], start[c+1]),
 * cell c = x + 32 y + 1024 z) and items[L] (input index of each listed primitive). */
int64_t mrt_regular_grid(const mrt_config *cfg, int32_t kind, float *world, int32_t *start, int32_t *items);
/* Host only: the membership test of a grid cell (Triangle::intersect(const AABB&),
 * Triangle.cpp:142-229; Plane.cpp:146-155; Sphere.cpp:102-123).  kind 0: prim = A, B, C xyz;
 * 1: point xyz, normal xyz; 2: center xyz, radius.  box = min xyz, max xyz.  1 / 0, or -1. */
int mrt_grid_box_test(int32_t kind, const float *prim, const float *box);
/* Host only: decode a map_Kd texture file as the renderer does (Texture::createTexture,
 * Texture.cpp:83-114: 8-bit channels with stb_image's conventions).  Returns the byte count
 * width*height*channels (and fills dims[3] = width, height, channels) or -1; with non-NULL
 * texels copies the image, row-major, channels interleaved. */
int64_t mrt_decode_texture(const char *path, int32_t *dims, uint8_t *texels);

/* Host only: the renderer's sample tables (2^20 floats each; trig: 2^21, cos and sin of
 * two_pi * shader[i] by the platform's libm, Shader.cpp:206-212).  NULL outputs are skipped. */
int mrt_sample_tables(float *shader, float *sampler, float *trig);

/* ---- test / diagnostic entry points (need a GPU; not on the render path) ----
 * Device known-answer tests: the slab test the trace kernels inline (AABB.cpp:34-54) on n
 * (box, ray) pairs: out[3i] = reference predicate, out[3i+1] = the IEEE min/max form used for
 * waves whose 1/d is finite, out[3i+2] = whether 1/d is finite.  boxes: n x (min xyz, max xyz). */
int mrt_kat_slab(const float *boxes, const float *orig, const float *dir, int32_t n, int32_t *out);
/* Triangle::intersect (Triangle.cpp:63-109) as the kernels evaluate it: tris n x (A, B, C) xyz;
 * hit[i] = 1 and t[i] on an accepted hit (eps <= t < RayLengthMax). */
int mrt_kat_triangle(const float *tris, const float *orig, const float *dir, int32_t n, int32_t *hit, float *t);
/* Arbitrary rays through the renderer's trace kernels (current walk and cull settings):
 * any = 0: closest hit (Shader::rayTrace intersection part, Shader.cpp:86-111): kind / index
 *          (input order, -1 on miss) / t per ray;
 * any = 1: Shader::shadowTrace (Shader.cpp:132-158) with tmax dist[i]: kind[i] = occluded.
 * src: NULL or n pairs (kind, input index) of the primitive each ray leaves (self-exclusion). */
int mrt_trace_rays(mrt_renderer *r, const float *orig, const float *dir, const float *dist, const int32_t *src,
                   int32_t n, int32_t any, int32_t *kind, int32_t *index, float *t);

#ifdef __cplusplus
}
#endif

#endif /* MOBILERT_AMD_H */
