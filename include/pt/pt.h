/*
 * pt.h -- C-ABI drop-in boundary of the MI355X path tracer (libpt.so).
 *
 * The reference has no C ABI: its boundary is the C++ scene API of namespace
 * PathTrace plus the templates tracePixel<T>/traceRay<T>.
 * Every entry point below replaces one reference interface, cited per line.
 * Plain pointers and sizes only; no exceptions cross the ABI: functions return
 * a status (PT_OK = 0, negative on error) or an id (>= 0, negative on error),
 * and pt_last_error() describes the last failure on the calling thread.
 *
 * Ownership mirrors the reference: a scene owns every texture, material,
 * object and image created in it; ids stay valid until pt_scene_destroy.
 * Objects may be referenced by several parents (the reference would
 * duplicate() them), materials are shared by reference as in the reference
 * (`const Material *`, include/sphere.h:12).
 *
 * Threading: a pt_scene may be rendered from one thread at a time; distinct
 * scenes are independent.  Rendering is synchronous unless pt_render_device
 * is given a stream.
 */
#ifndef PT_PT_H
#define PT_PT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_OK 0
#define PT_ERR_ARG (-1)      /* bad id / argument (reference: assert or UB)          */
#define PT_ERR_MATH (-2)     /* singular matrix: std::domain_error, transform.h:353   */
#define PT_ERR_IO (-3)       /* ImageLoadError / ImageStoreError, image.h:30-46       */
#define PT_ERR_DEVICE (-4)   /* HIP runtime failure or no device                      */
#define PT_ERR_COMPILE (-5)  /* device code generation / hiprtc failure               */

typedef struct pt_scene pt_scene;
typedef int32_t pt_id;

/* ------------------------------------------------------------ lifetime -- */
pt_scene *pt_scene_create(void);
void pt_scene_destroy(pt_scene *s);
const char *pt_last_error(void);
const char *pt_version(void);

/* ------------------------------------------------------------- images --- */
/* Image(string fileName) for ".hdr"/".pic" (reference src/image.cpp:83-324). */
pt_id pt_image_load_hdr(pt_scene *s, const char *path);
/* Image(string fileName) for ".png": PngDecoder (reference src/png_decoder.cpp:
 * 40-128) + byte / 255.0f (src/image.cpp:60-79); RGB gets alpha 0 (the
 * png_set_filler(0) of :94-97), palette tRNS becomes alpha.  Grayscale PNGs
 * are PT_ERR_IO (the reference's decoder leaves their rows half written). */
pt_id pt_image_load_png(pt_scene *s, const char *path);
/* Image(string fileName) with the format taken from the extension
 * (src/image.cpp:49-59): "png", "hdr", "pic" (case-insensitive). */
pt_id pt_image_load(pt_scene *s, const char *path);
/* MutableImage -> Image (include/image.h:110-211): rgba is h rows of w RGBA
 * floats, row 0 = top; copied. */
pt_id pt_image_from_rgba32f(pt_scene *s, const float *rgba, int w, int h);
/* Decode a Radiance HDR file into caller memory (w*h*4 floats); pass
 * rgba=NULL to query the size. */
int pt_hdr_read(const char *path, float *rgba, int *w, int *h);
/* The same for a PNG file (pt_image_load_png's decoding). */
int pt_png_read(const char *path, float *rgba, int *w, int *h);

/* ----------------------------------------------------------- textures --- */
pt_id pt_tex_color(pt_scene *s, float r, float g, float b);              /* ColorTexture       texture.h:29-58  */
pt_id pt_tex_image(pt_scene *s, pt_id image);                            /* ImageTexture       image_texture.h:9-33 */
pt_id pt_tex_image_alpha(pt_scene *s, pt_id image);                      /* ImageAlphaTexture  image_texture.h:35-70 */
pt_id pt_tex_skybox(pt_scene *s, pt_id top, pt_id bottom, pt_id left,    /* ImageSkyboxTexture image_texture.h:72-115 */
                    pt_id right, pt_id front, pt_id back);
pt_id pt_tex_skybox_alpha(pt_scene *s, pt_id top, pt_id bottom, pt_id left, /* ImageSkyboxAlphaTexture :117-181 */
                          pt_id right, pt_id front, pt_id back);
pt_id pt_tex_multiply(pt_scene *s, float r, float g, float b, pt_id t);  /* MultiplyTexture    filter_texture.h:36-56 */
pt_id pt_tex_log(pt_scene *s, pt_id t);                                  /* LogTexture         filter_texture.h:58-82 */
pt_id pt_tex_mirrorball(pt_scene *s, pt_id t);                           /* MirrorBallSkymapTexture transform_texture.h:33-59 */
pt_id pt_tex_spherical(pt_scene *s, pt_id t);                            /* SphericalCoordinatesSkymapTexture :61-85 */
pt_id pt_tex_transformed(pt_scene *s, const float m[12], pt_id t);      /* TransformedTexture texture.h:60-90 */
pt_id pt_tex_coord(pt_scene *s);                                         /* test instrument: colour = coordinate */
/* A user-defined Texture subclass (include/texture.h:10-27: the virtual
 * getColor, and getFloat unless it keeps the default mean of getColor) as
 * device source.  color_body is the body of
 *     V3 getColor(V3 p)           -- p.x, p.y, p.z: the lookup point
 * and value_body (NULL = the reference's default) the body of
 *     float getFloat(V3 p)
 * in the device library's vocabulary (V3, mk(x, y, z), the f32 math builtins
 * floorf, fabsf, sqrtf, fminf, ...); both read their nparams parameters as
 * `const float *prm`.  The bodies are compiled into every module of the scene
 * that reaches the texture, with the scene's options: no FMA contraction and
 * correctly rounded '/' and sqrt, so a body computes what the same text
 * compiled on the host with -ffp-contract=off computes.  A body that does not
 * compile makes the render fail with PT_ERR_COMPILE and the compiler's log in
 * pt_last_error(). */
pt_id pt_tex_device(pt_scene *s, const char *color_body, const char *value_body, const float *params, int nparams);

/* ---------------------------------------------------------- materials --- */
/* Material(reflect, scatter_coefficient, emissive, transmit, ior,
 * transmit_reflect_coefficient), include/material.h:18.  Pass -1 for a
 * texture to get the reference default (1, 1, 0, 0, -, 0). */
pt_id pt_material(pt_scene *s, pt_id reflect, pt_id scatter, pt_id emissive, pt_id transmit, float ior,
                  pt_id transmit_reflect);

/* ------------------------------------------------------------ objects --- */
pt_id pt_sphere(pt_scene *s, float cx, float cy, float cz, float r, pt_id mat);   /* Sphere  sphere.h:12 */
pt_id pt_plane(pt_scene *s, float nx, float ny, float nz, float d, pt_id mat);    /* Plane(n, d)   plane.h:12 */
pt_id pt_plane_through(pt_scene *s, float nx, float ny, float nz,                 /* Plane(n, pos) plane.h:13 */
                       float px, float py, float pz, pt_id mat);
#define PT_CSG_UNION 0        /* Union        union.h:12        */
#define PT_CSG_INTERSECTION 1 /* Intersection intersection.h:12 */
#define PT_CSG_DIFFERENCE 2   /* Difference   difference.h:12   */
pt_id pt_csg(pt_scene *s, int op, pt_id a, pt_id b);
pt_id pt_transformed(pt_scene *s, const float m[12], pt_id child);             /* TransformedObject object.h:78 */
/* A user-defined Object subclass (include/object.h:10-24: the virtual
 * makeSpanIterator) whose iterator yields at most one span per ray -- a convex
 * shape -- as device source, compiled into the scene's modules
 * (path-trace_amd/csrc/device/pt_user_object.h).  span_body is the body of
 *     bool span(V3 o, V3 d, float &t0, float &t1)
 * returning whether the ray o + t d (d not normalised) meets the object, and
 * then its entry and exit parameters t0 <= t1 (the Span's start and end,
 * include/span.h); normal_body is the body of
 *     V3 normal(V3 p)
 * returning the outward surface normal at p, which is the span's start normal
 * at the entry point and its end normal at the exit.  Both read the nparams
 * parameters as `const float *prm` and use the device library's vocabulary
 * (V3, mk, dot, normalize, the f32 math builtins), compiled without FMA
 * contraction and with correctly rounded '/' and sqrt, so they compute what
 * the same text compiled on the host with -ffp-contract=off computes.  The
 * object takes part in every CSG node and transform like a built-in
 * primitive; the kernel's fast paths treat it conservatively (never dark). */
pt_id pt_object_device(pt_scene *s, const char *span_body, const char *normal_body, const float *params,
                       int nparams, pt_id mat);
int pt_set_root(pt_scene *s, pt_id obj);
/* Load a whole scene from the plain-text scene format (oracle/scene_text.h
 * documents it; pathtrace.scene.to_text writes it).  Replaces the current
 * contents of s. */
int pt_scene_from_text(pt_scene *s, const char *text);

/* ---------------------------------------------------- matrix helpers --- */
/* Float arithmetic of include/transform.h:207-421, m in constructor order
 * x00 x10 x20 x30 x01 x11 x21 x31 x02 x12 x22 x32. */
void pt_matrix_rotate(const float axis[3], double angle, float out[12]);
int pt_matrix_inverse(const float m[12], float out[12]);                /* PT_ERR_MATH if singular */
void pt_matrix_concat(const float a[12], const float b[12], float out[12]);

/* ------------------------------------------------------------- render --- */
#define PT_ORDER_FAST 0      /* fast path: a burst's non-zero leaf-child terms dealt round-robin to 64
                                lane sums, added as their pairwise tree; samples in
                                32-sample pairwise blocks (oracle.cpp ORDER_FAST)     */
#define PT_ORDER_REFERENCE 1 /* bit-for-bit the reference's sequential child order          */
#define PT_ORDER_GROUP64 PT_ORDER_FAST /* deprecated name of PT_ORDER_FAST (rounds 1-2)      */

typedef struct pt_render_params {
    int width, height;             /* screenXResolution, screenYResolution                      */
    int spp;                       /* sampleCount                                               */
    int depth;                     /* rayDepth                                                  */
    float screen_w, screen_h;      /* screenWidth, screenHeight                                 */
    float screen_dist;             /* screenDistance                                            */
    uint64_t seed;                 /* run seed of the per-(pixel, sample) engine (pt_engine.h)  */
    int order;                     /* PT_ORDER_*                                                */
    int device;                    /* HIP device ordinal                                        */
    const int32_t *pixels;         /* optional host list of pixel indices (y*width+x) to render;
                                      NULL = all pixels                                         */
    int64_t npixels;               /* length of pixels                                          */
    int64_t max_buffer_bytes;      /* per-sample staging budget (0 = 8 GiB)                     */
    int grid_width;                /* pixel index = y * grid_width + x (0 = width); > width
                                      addresses pixels past the right / bottom edge, as the
                                      adaptive caller's block edges do                          */
    int sample_begin;              /* engine sample index of this call's first sample: the call
                                      renders samples sample_begin .. sample_begin + spp - 1 of
                                      each pixel (a rank's share when samples are split)        */
    int sum_only;                  /* nonzero: write each pixel's sum of those samples, in
                                      sample order, without the division by spp               */
} pt_render_params;

typedef struct pt_render_stats {
    double kernel_ms;              /* summed render-kernel time (HIP events)                    */
    double reduce_ms;              /* summed reduce-kernel time                                 */
    uint64_t launches;             /* render-kernel launches                                    */
    uint64_t samples;              /* traceRay calls from tracePixel                            */
    uint64_t queries;              /* root span queries (spine + leaf children)                 */
    uint64_t leaf_queries;         /* of which wave-cooperative leaf children                   */
    uint64_t attempts;             /* rejection attempts consumed (a round evaluates 512)       */
    uint64_t rounds;               /* attempt rounds                                            */
    uint64_t sphere_tests, sphere_hits, plane_tests;
    uint64_t slow_queries;         /* leaf children that needed the full CSG merge (slow pass)  */
    uint64_t dark_queries;         /* leaf children no emissive primitive can light: weight * 0 */
    uint64_t mid_queries;          /* leaf children the clear pass could not finish (fast check) */
    double wave_ms;                /* mean render-wave lifetime (device clock); kernel_ms minus
                                      this is the launch's tail, where waves have run out of work */
} pt_render_stats;

/* Synchronous: renders the frame into rgb_out (host memory), which receives,
 * for each pixel of params->pixels (or of the whole frame, row-major), the
 * mean radiance (r, g, b) exactly as tracePixel returns it (path-trace.h:187-201).
 * Replaces the per-pixel tracePixel calls of RenderBlock::calcPixelColor
 * (reference src/test.cpp:441-465).  stats = NULL skips the launches' timing
 * events and the counter read-back (the per-pixel caller's fast path). */
int pt_render(pt_scene *s, const pt_render_params *p, float *rgb_out, pt_render_stats *stats);

/* The multi-GPU partition (replaces the reference's TCP block farm,
 * src/test.cpp:520-778): the pixel indices (y * width + x, raster order) rank
 * `rank` of `world` renders in the lattice deal of tile x tile tiles -- tile
 * (tx, ty) belongs to rank (tx + 3 ty) mod world -- the default of bench.py
 * and pathtrace.dist.rank_pixels.  Every pixel has exactly one owner, so the
 * ranks' frames (pt_render_device with the list into a zeroed full frame)
 * sum to the one-GPU frame bit for bit.  pixels = NULL: *count receives the
 * number only; else at most capacity indices are written. */
int pt_rank_pixels(int width, int height, int rank, int world, int tile, int32_t *pixels, int64_t capacity,
                   int64_t *count);

/* Host-clock phases (microseconds) of the calling thread's last pt_render --
 * the breakdown of a per-pixel tracePixel call.  out[k]
 * for k < n: */
#define PT_PROF_TOTAL 0   /* the whole call                                                   */
#define PT_PROF_SETUP 1   /* validation, the scene's generated module (cached), device buffers */
#define PT_PROF_ENQUEUE 2 /* pixel upload, counter reset, render + reduce launches, the
                             result's copy-back (with stats: also the wait for the
                             launches' timing events)                                       */
#define PT_PROF_WAIT 3    /* stream synchronise: the kernels' remaining run time and the
                             copy-back (results up to 4 MB: a DMA into pinned staging)       */
#define PT_PROF_D2H 4     /* the result into the caller's memory (pinned staging: a memcpy;
                             larger results: a synchronous device-to-host copy)              */
#define PT_PROF_KERNEL 5  /* render launch(es) by HIP events (0 unless stats were asked for,
                             or PT_CALL_KERNEL_TIME is set)                                   */
#define PT_PROF_REDUCE 6  /* pt_reduce by HIP events (the same condition)                     */
#define PT_PROF_N 7
int pt_call_profile(double *out, int n);

/* Device variant: writes W*H*3 floats into device memory fb (full frame,
 * row-major; with params->pixels, 3 floats at 3*index for every listed index,
 * so fb must cover the largest one; other pixels are left untouched) on the
 * given hipStream_t (NULL = default stream) and returns once the work is
 * enqueued... or completed when stats != NULL (stats need the timings). */
int pt_render_device(pt_scene *s, const pt_render_params *p, float *fb, void *stream, pt_render_stats *stats);

/* pt_render_device that stays asynchronous and still keeps its timings: HIP
 * events around each launch and the device counters accumulate on the scene's
 * device until pt_render_collect, so a caller can queue the render, a
 * collective on the same stream and more renders without a host round trip
 * (bench.py's multi-GPU step: render, then the RCCL reduce of the frame).
 * At most 1024 timed renders may wait for a collect (PT_ERR_ARG after that).
 * An untimed pt_render_device queued while timed renders wait joins them: its
 * launches are timed and its counters go into the next collect's totals, and
 * it never counts against the cap. */
int pt_render_device_timed(pt_scene *s, const pt_render_params *p, float *fb, void *stream);

/* Waits for the timed renders queued on `device` since the last collect and
 * returns their summed statistics (kernel_ms, launches, samples, counters);
 * all zero when none are pending. */
int pt_render_collect(pt_scene *s, int device, pt_render_stats *stats);

/* The reference demo's image-formation policy, RenderBlock::renderSquare
 * (src/test.cpp:423-507): per block of block_size x block_size pixels, trace
 * the corners, then recursively either interpolate a square (size <=
 * max_interp and all six corner pairs within min_delta: colorCloseEnough,
 * :437-440, interpolateSquare :423-436) or trace its five subdivision points
 * and recurse into the quadrants.  Pixels are traced with p->spp samples each,
 * one GPU batch per subdivision level over all blocks; engine keys use the
 * grid y * gw + x with gw = ceil(width / block) * block + 1 (block corners
 * reach past the right edge).  rgb_out receives
 * the W*H*3 image.  block_size / max_interp <= 0 select the demo's values
 * (getBlockSize(width / 8), height / 120, :40-50); min_delta <= 0 selects 0.003. */
typedef struct pt_adaptive_params {
    int block_size;
    int max_interp;
    float min_delta;
    int64_t traced_pixels;         /* out: pixels traced whose colour the image used            */
    int levels;                    /* out: GPU batches                                          */
    int exact_batches;             /* in: nonzero = one batch per level, only needed points     */
    int64_t lookahead_pixels;      /* out: traced one level ahead and never used                */
} pt_adaptive_params;
int pt_render_adaptive(pt_scene *s, const pt_render_params *p, pt_adaptive_params *ap, float *rgb_out,
                       pt_render_stats *stats);

/* traceRay<T>(const Ray &ray, SpanIterator &, int depth, T &engine, float
 * strength) of include/path-trace.h:58-165 for a batch of caller rays, in one
 * device launch.  rays = n records of 7 floats: origin xyz, direction xyz
 * (non-zero: Ray's assert, include/ray.h:17; not normalised), strength.
 * Origin and direction components must be finite (PT_ERR_ARG otherwise): the
 * kernel's axis-aligned plane forms keep only the product that is non-zero for
 * finite operands, where the reference's full dot product of an infinite
 * component would be NaN.
 * rgb_out receives, per ray, the mean of spp traceRay samples -- sample s of ray
 * k drawing from the engine keyed (seed, ray_begin + k, sample_begin + s), include/pt/
 * pt_engine.h -- summed in `order` and divided by spp: with spp = 1 the
 * traceRay value itself (as (0 + c) / 1: a -0 channel reads +0), with the
 * camera ray of a point and spp = sampleCount tracePixel's float-coordinate
 * overload (path-trace.h:172-185). */
typedef struct pt_trace_params {
    int spp;                       /* samples per ray (>= 1)                                    */
    int depth;                     /* rayDepth                                                  */
    uint64_t seed;                 /* run seed of the per-(ray, sample) engine                  */
    int order;                     /* PT_ORDER_*                                                */
    int device;                    /* HIP device ordinal                                        */
    int sample_begin;              /* engine sample index of the first sample                   */
    int64_t max_buffer_bytes;      /* per-sample staging budget (0 = 8 GiB)                     */
    int64_t ray_begin;             /* engine key index of rays[0] (ray k: ray_begin + k), so
                                      successive calls can draw fresh streams                  */
} pt_trace_params;
int pt_trace_rays(pt_scene *s, const pt_trace_params *p, const float *rays, int64_t n, float *rgb_out,
                  pt_render_stats *stats);
/* JIT-compile (or fetch from the cache) pt_trace_rays' module for this scene
 * and depth without touching a GPU. */
int pt_trace_compile(pt_scene *s, int depth);

/* Everything a render with p needs -- code object loaded, scene parameters
 * and images uploaded, staging buffers allocated -- without rendering, so a
 * timed or latency-sensitive render does no compilation or allocation. */
int pt_prepare(pt_scene *s, const pt_render_params *p);

/* JIT-compile (or fetch from the code-object cache) the megakernel for this
 * scene and depth without touching a GPU.  Used by build() to pre-populate the
 * in-tree cache. */
int pt_scene_compile(pt_scene *s, int depth);
/* MI355X tuning knob, no reference counterpart: build this scene's megakernel
 * for 1..5 resident workgroups (of 4 waves) per CU instead of the most its
 * LDS allows (0 = auto).  Fewer workgroups raise the VGPR cap (5: 96, 4: 128,
 * 3: 168, 2: 256): scenes whose CSG tree spills at the default cap and whose
 * samples are mostly spine walks run faster (C5: 2.3x at 2), burst-bound
 * scenes slower (C2 at 2: -8 %).  Takes effect at the next compile/render. */
int pt_scene_set_occupancy(pt_scene *s, int workgroups_per_cu);
/* MI355X tuning knob, no reference counterpart: the wave-walked (spine) and
 * lane-walked (camera, lane-finished child) queries of this scene first take
 * every primitive's span and the fast checks, and run the lazy merge only
 * where those cannot decide (same bits either way).  Pays where rays rarely
 * start inside overlapping CSG spans (C5: 288 -> 568 Msamples/s), costs
 * where they often do (C3 spine: -0.9 %).  Takes effect at the next
 * compile/render. */
int pt_scene_set_fast_spine(pt_scene *s, int on);
/* MI355X tuning knob, no reference counterpart: each lane of a chunk walks its
 * own sample's ray tree when no node of it has a scatter loop (mirrors, glass,
 * emitters), with `frames` (1..8) register frames for pending nodes; samples
 * that need a scatter loop or a deeper stack go to the wave as before (same
 * bits either way).  Pays where such trees are common (C5's glass ball), costs
 * registers elsewhere.  0 = off.  Takes effect at the next compile/render. */
int pt_scene_set_lane_walk(pt_scene *s, int frames);
/* MI355X tuning knob, no reference counterpart: each lane of a chunk walks its
 * own sample's whole ray tree, scatter loops included, drawing its engine's
 * numbers one rejection attempt after another; loops of more than 64 children
 * that mostly end in leaves (a plain diffuse bounce) and fast-order runs of
 * more than 64 non-zero terms go to the wave as before (same bits either way).
 * Pays where scatter loops are small or recurse often (C2's
 * matBrightDiffuseWhite: ~10^4 children, a quarter of them recursing into a
 * dozen leaves each); supersedes pt_scene_set_lane_walk.  Takes effect at the
 * next compile/render. */
int pt_scene_set_lane_scatter(pt_scene *s, int on);
/* MI355X tuning knob, no reference counterpart: lane-walk scenes render in
 * split launches (default on) -- a light kernel (no lazy merges, no wave walk,
 * higher occupancy) over every chunk, then the full kernel over the chunks
 * with a lane it could not finish.  A chunk's sums come from one kernel, so
 * the bits are the same either way.  0 = every chunk through the full kernel.
 * Takes effect at the next render. */
int pt_scene_set_split(pt_scene *s, int on);
/* Key of the code object for this scene/depth: a hash of the generated source,
 * the compiler options and the hiprtc version -- the file name of its entry in
 * the code-object cache (hex string, thread-local storage). */
const char *pt_scene_kernel_key(pt_scene *s, int depth);

/* ------------------------------------------------------------ queries --- */
/* The reference's query virtuals, evaluated on the device.
 *
 * pt_query_spans: obj->makeSpanIterator() (include/object.h:14), then for each
 * ray (6 floats: origin xyz, direction xyz) init(ray) and next() until
 * isAtEnd() (include/span.h:129-171).  counts[i] receives ray i's number of
 * spans; the first min(counts[i], max_spans) spans go to out[i * max_spans ..]
 * in the reference's Span form (span.h:12-120; materials as pt_ids).  obj < 0
 * queries the scene root.  The lists are bit-identical to the reference's,
 * including the Difference quirk (src/difference.cpp:124-130). */
typedef struct pt_span {
    float t_start, n_start[3];     /* start, startNormal   */
    int32_t mat_start;             /* startMaterial        */
    float t_end, n_end[3];         /* end, endNormal       */
    int32_t mat_end;               /* endMaterial          */
} pt_span;
int pt_query_spans(pt_scene *s, pt_id obj, const float *rays, int64_t n, int max_spans, pt_span *out,
                   int32_t *counts, int device);
/* Texture::getColor (rgb: 3 floats per point) and Texture::getFloat (value: 1
 * float per point) of texture tex at n points (3 floats each),
 * include/texture.h:13-18 with every subclass's override. */
int pt_tex_eval(pt_scene *s, pt_id tex, const float *points, int64_t n, float *rgb, float *value, int device);
/* Compile (or fetch from the code-object cache) the query module of obj
 * (-1: the root, when tex < 0; -2: none) and/or tex (-1: none), without a
 * device. */
int pt_query_compile(pt_scene *s, pt_id obj, pt_id tex);

/* Device self-test: the megakernel's exact fast paths for f32 sqrt / '/' /
 * normalize against the compiler's correctly rounded ones on n hashed inputs.
 * mismatches[0..2] receive the sqrt, div and normalize mismatch counts. */
int pt_selftest_math(int device, uint64_t n, uint64_t seed, uint64_t *mismatches);

/* Device self-test of the restated glibc float libm the texture maps use
 * (SphericalCoordinatesSkymapTexture's atan2f / asinf, transform_texture.h:
 * 73-85; LogTexture's logf, filter_texture.h:62-67): for n operand pairs
 * ops[2i] = y, ops[2i+1] = x, out[3i..3i+2] = atan2f(y, x), asinf(y), logf(x)
 * as the device computes them, for comparison with the host's libm. */
int pt_selftest_libm(int device, const float *ops, int64_t n, float *out);

/* ------------------------------------------------------------- output --- */
/* MutableImage::writeHDR (reference src/image.cpp:398-481), rgb = w*h*3 floats. */
int pt_write_hdr(const char *path, const float *rgb, int w, int h);
/* 24-bpp BGR bottom-up BMP as SDL_SaveBMP writes it, bytes
 * clamp(floor(256*c/count), 0, 255) (reference src/test.cpp:1037-1059). */
int pt_write_bmp(const char *path, const float *rgb, int w, int h, int count);

#ifdef __cplusplus
}
#endif

#endif
