/*
 * vxpt -- C ABI of the MI355X-native voxel path-tracing hot path.
 *
 * Drop-in boundary for the reference's offline render path
 * (mainOffline.cpp -> OfflineBackend::renderFrame, OfflineBackend.cpp:46-89).
 * The reference's entry points are C++ singletons with no ABI; each function
 * below names the reference interface it replaces.
 *
 * Conventions: every call returns 0 on success or a negative vxpt_status;
 * vxpt_last_error() returns a message for the last failure on that context.
 * No exceptions cross this boundary.  One context per GPU; calls on one
 * context are not thread safe.  All work is enqueued on the context's HIP
 * stream; vxpt_sync() waits for it.  Host pointers are plain host memory.
 */
#ifndef VXPT_H
#define VXPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vxpt_ctx vxpt_ctx;

enum vxpt_status {
    VXPT_OK = 0,
    VXPT_ERR_ARG = -1,
    VXPT_ERR_HIP = -2,
    VXPT_ERR_IO = -3,
    VXPT_ERR_STATE = -4,
    VXPT_ERR_NODEV = -5
};

/* Logical per-pixel buffers (BufferManager.cpp:150-206).  float4 planes are
 * W*H*16 B, float planes W*H*4 B, RESERVOIRS is 2*W*H*20 B (both parities). */
enum vxpt_buffer {
    VXPT_BUF_ILLUM = 0, VXPT_BUF_DEPTH = 1, VXPT_BUF_NORMAL_ROUGH = 2, VXPT_BUF_GEO_NORMAL_THIN = 3,
    VXPT_BUF_ALBEDO = 4, VXPT_BUF_MATERIAL = 5, VXPT_BUF_MAT_PARAM = 6, VXPT_BUF_MOTION = 7,
    VXPT_BUF_PREV_NORMAL_ROUGH = 8, VXPT_BUF_PREV_GEO_NORMAL_THIN = 9, VXPT_BUF_PREV_ALBEDO = 10,
    VXPT_BUF_PREV_MAT_PARAM = 11, VXPT_BUF_PREV_DEPTH = 12, VXPT_BUF_PREV_MATERIAL = 13,
    VXPT_BUF_RESERVOIRS = 14, VXPT_BUF_PING = 15, VXPT_BUF_PONG = 16, VXPT_BUF_PREV_ILLUM = 17,
    VXPT_BUF_PREV_FAST = 18, VXPT_BUF_HIST_LEN = 19, VXPT_BUF_PREV_HIST_LEN = 20, VXPT_BUF_OUTPUT = 21,
    VXPT_BUF_SKY = 32,       /* 1024*512 float4 sky map (Sky.cu:259-303)      */
    VXPT_BUF_SUN = 33,       /* 32*32 float4 sun map (Sky.cu:305-327)          */
    VXPT_BUF_VOXELS = 34,    /* chunk-major u8 block ids                        */
    VXPT_BUF_RES_EVEN = 35,  /* reservoirs of even iterationIndex (W*H*20 B)   */
    VXPT_BUF_RES_ODD = 36,   /* reservoirs of odd iterationIndex               */
    VXPT_BUF_WPOS = 37,      /* per-pixel hit world position (denoiser)        */
    VXPT_BUF_FRAME = 38,     /* post-processed frame, Float4(sRGB, 0) (OfflineBackend m_frameBuffer) */
    /* traversal structures (read-only parity hooks for the incremental edit path) */
    VXPT_BUF_OCTANT_TABLES = 39, /* 8 x nBricks u8: empty-cube edge per brick and ray octant  */
    VXPT_BUF_CELL_MASKS = 40,    /* nBricks u64: cube-cell bits of each 4^3 brick             */
    VXPT_BUF_BRICK_IDS = 41,     /* nBricks x 64 u8: ids in brick-major order                 */
    VXPT_BUF_MACRO_MASKS = 42,   /* nBricks/64 u64: occupied-brick bits of each 16^3 cell      */
    VXPT_BUF_TEXELS = 43,        /* every loaded texture's RGBA8 mip chain (vxpt_texture_table) */
    /* emissive-triangle lights of the instanced meshes (vxpt_load_models / vxpt_get_lights) */
    VXPT_BUF_LIGHTS = 44,        /* nLights x 32 B LightInfo (Light.h:13-23)                     */
    VXPT_BUF_LIGHT_ALIAS = 45,   /* nLights x {f32 q, f32 p, i32 alias} (AliasTable.h bins)      */
    VXPT_BUF_BLOOM = 46,         /* post-process: the horizontally blurred bloom, Float4 per pixel */
    VXPT_BUF_TAP_RECORD = 47,    /* read-only: the last pass's ReSTIR tap records, 32 B per pixel (normal xyz,
                                  * roughness with the metallic flag in its sign bit; albedo xyz, depth) --
                                  * the G-buffer planes GetPrevSurface reads (Restir.h:348-381), packed */
    VXPT_BUF_BOX_TABLES = 48,    /* read-only: 8 x nBricks u32, the walk's empty-box extents per brick and ray
                                  * octant (x | y << 8 | z << 16 bricks; 0 = occupied), box_tables.hpp */
    VXPT_BUF_CLAMP_DECISION = 49 /* read-only parity hook (vxpt_debug_clamp_decisions): per pixel, a float
                                  * holding the last denoise's history-clamp decision bits -- 1: the x-only
                                  * Float3 compare cmin.x < centre.x (HistoryClamping.h:124), 2: cmax.x >
                                  * centre.x (:125), 4: the pixel's history exceeds 4 frames, so the clamp
                                  * uses them, 8: its anti-lag factor's quotient (:131) is ill-conditioned
                                  * (denominator within 1e-3 of the luma, quotient inside (0, 1)); 0 where
                                  * the clamp did not run */
};

typedef struct vxpt_config {
    int32_t width, height;   /* frame size, any positive size.  The reference's Atrous has no bounds guard:
                                 its threads past a frame edge store to the clamped edge pixels (a race
                                 when the size is not a multiple of 16); here those threads are masked */
    int32_t device;          /* HIP device ordinal                                                */
    int32_t row_begin, row_end; /* band of rows this context traces (multi-GPU); 0,0 = all      */
    int32_t total_bounce_limit;   /* RayGen.cu:146 (3)  */
    int32_t diffuse_bounce_limit; /* RayGen.cu:147 (1)  */
    const char *data_dir;    /* directory holding tables/, settings/, scene/, assets/             */
} vxpt_config;

typedef struct vxpt_camera {
    float pos[3];
    float dir[3];            /* scene_export.yaml camera.direction (normalised internally) */
    float fov_deg;           /* horizontal field of view                                   */
} vxpt_camera;

typedef struct vxpt_material {
    float albedo[3];
    float roughness;
    float translucency;
    int32_t metallic;
    int32_t material_id;     /* MaterialParameter.materialId, written to the material G-buffer */
    int32_t thinfilm;
} vxpt_material;

typedef struct vxpt_denoise_params { /* DenoisingParams, GlobalSettings.h:82-141 */
    float max_accumulated_frame_num, max_fast_accumulated_frame_num, phi_luminance;
    float lobe_angle_fraction, roughness_fraction, depth_threshold;
    float disocclusion_threshold, disocclusion_threshold_alternate, denoising_range;
    int32_t enable_temporal_accumulation, enable_history_fix, enable_history_clamping;
    int32_t enable_spatial_filtering, enable_firefly_filter, atrous_iteration_num;
} vxpt_denoise_params;

typedef struct vxpt_post_params { /* ToneMappingParams + PostProcessingPipelineParams (GlobalSettings.h:10-186),
                                      yaml section `postprocess` */
    float manual_exposure;
    int32_t tone_mapping_curve;      /* 0 Narkowicz ACES, 1 Uncharted 2, 2 Reinhard */
    float white_point, contrast, saturation, lift, gain;
    int32_t enable_bloom;
    float bloom_threshold, bloom_intensity, bloom_radius;
    int32_t enable_auto_exposure;
    float exposure_speed, exposure_min, exposure_max, exposure_compensation;
    float histogram_min_percent, histogram_max_percent, target_luminance;
    int32_t enable_vignette;
    float vignette_strength, vignette_radius, vignette_smoothness;
    int32_t enable_lens_flare;
    float lens_flare_intensity, lens_flare_ghost_spacing;
    int32_t lens_flare_ghost_count;
    float lens_flare_halo_radius, lens_flare_sun_size, lens_flare_distortion;
    int32_t draw_crosshair;          /* DrawCrosshair (PostProcessor.cu:14-46), on in the reference */
} vxpt_post_params;

typedef struct vxpt_image_diff_result { /* ImageDiffResult (renderer/util/ImageDiff.h:7-26) */
    int32_t total_pixels, different_pixels;
    float pixel_difference_ratio, rmse, ssim;
    int32_t is_identical, is_very_close, is_close;
} vxpt_image_diff_result;

typedef struct vxpt_timing {  /* HIP-event times of the last frame, ms (replaces PerformanceTracker) */
    float trace_ms;
    float denoise_ms;
    float sky_ms;
    float frame_ms;
    float host_ms;  /* host time per frame to enqueue the last vxpt_render_frames run (before its final sync):
                       close to frame_ms means the GPU waited for the host */
} vxpt_timing;

/* Schedule and traversal tuning of a context (no reference counterpart: the reference's OptiX
 * launch has no such knobs).  No field changes a result, only how long a frame takes; the defaults
 * (vxpt_tuning_defaults) are the measured best.  The library reads no
 * environment variable: this struct is the only way to change its schedule. */
typedef struct vxpt_tuning {
    int32_t dda_boxes;        /* 1: the walk skips empty space with empty-box tables; 0: cube tables   (1) */
    int32_t box_cap;          /* box growth limit in bricks, sideways octants, 1..255                  (32) */
    int32_t box_cap_up;       /* the same for the upward octants                                       (32) */
    int32_t brick_steps;      /* in-brick cell crossings before a queued walk yields, 1..64            (3) */
    int32_t cam_steps;        /* the same for camera / continuing path rays (k_closest), 1..64         (10) */
    int32_t iter_cap;         /* outer walk iterations before a queued ray becomes a straggler, 1..1024 (4) */
    int32_t iter_cap2;        /* a second straggler level after that many more (0: off), 0..1024      (6) */
    int32_t resume_wg_per_cu; /* straggler-resume workgroups per CU, 1..64                              (24) */
    int32_t sort_mode;        /* queued rays grouped per workgroup: 0 off, 1 octant, 2 octant x axis    (2) */
    int32_t overlap;          /* 1: pass halves and pipelined frames on two streams; 0: in order        (1) */
    int32_t state_sets;       /* wavefront state sets, 2..3: a pass's first half waits for the second half
                                 state_sets passes back                                                (3) */
    int32_t firefly_fused;    /* 1: the detecting wave filters its fireflies; 0: a second launch        (1) */
    int32_t ta_supertiles;    /* 1: temporal accumulation on XCD supertiles; 0: raster tiles            (1) */
    int32_t hf_split;         /* history-fix workgroups per tile, 1..16                                 (4) */
    int32_t stencil_tile;     /* tile edge of the history clamp and the first a-trous, 16 or 32        (16) */
    int32_t front_streams;    /* streams for the passes' first halves (by state set), 1..3: side by side (2) */
    int32_t lds_bricks;       /* 1: camera walks read bricks through a workgroup cache in LDS           (0) */
    int32_t resume_split;     /* the last straggler level's walks cut into 1, 2, 4, 8 or 16 pieces walked
                                 side by side                                                          (16) */
    int32_t later_split;      /* the later path segments' stragglers: after 8 more iterations, in 1-16 pieces (16) */
    int32_t restir_waves;     /* k_restir's occupancy: 0 the compiler's register budget (3 waves/SIMD), 4: bounded
                                 to 4 waves (spills; a small band's launch fits one generation of waves)   (0) */
    int32_t ghost_rows;       /* banded frames: 1: the history clamp and the a-trous steps compute the rows they
                                 read outside the band (2 exchanges in the chain instead of 6); 0: exchange
                                 after every pass                                                          (1) */
    int32_t chain_gate;       /* pipelined frames (vxpt_render_frames, banded frames): 1: a frame's later passes'
                                 first halves are enqueued once the previous frame's denoiser chain has
                                 finished (the chain runs alone); 0: as soon as their state set is free
                                 (spp >= 2 and no uploaded motion plane; otherwise the gate stays)       (1) */
    int32_t sky_exit;         /* 1: a walk that leaves an empty box above the world's highest cube cell without
                                 heading down ends there (nothing ahead can be hit)                      (1) */
    int32_t xcd_order;        /* XCD-local work order, bits: 1 k_restir and 2 k_closest take their pixel tiles in
                                 XCD-local panels (each XCD one stripe of tile rows, walked column by
                                 column: the temporal taps / bricks of the workgroups in flight on one XCD
                                 meet in its L2); 4 k_queue's workgroups take one contiguous run of the
                                 queue per XCD; 0: raster / queue order, 0..7                             (0) */
    int32_t iter_cap3;        /* with iter_cap2: a third straggler level after iter_cap2 more iterations, the
                                 level-2 walks resumed for that many more before the last level (0: off),
                                 0..1024                                                                 (12) */
    int32_t iter_cap4;        /* with iter_cap3: a fourth level, the level-3 walks resumed for that many more
                                 before the last level (0: off), 0..1024                                   (0) */
} vxpt_tuning;
int vxpt_tuning_defaults(vxpt_tuning *out);
int vxpt_get_tuning(vxpt_ctx *ctx, vxpt_tuning *out);
/* between frames; dda_boxes / box caps rebuild the current world's skip tables (VXPT_ERR_ARG for a
 * field out of range, nothing changed then) */
int vxpt_set_tuning(vxpt_ctx *ctx, const vxpt_tuning *t);

/* replaces OfflineBackend::init(w,h) + BufferManager::init (OfflineBackend.h:30, BufferManager.cpp:107) */
int vxpt_create(const vxpt_config *cfg, vxpt_ctx **out);
/* replaces OfflineBackend::clear (OfflineBackend.h:31) */
void vxpt_destroy(vxpt_ctx *ctx);
const char *vxpt_last_error(const vxpt_ctx *ctx);

/* GlobalSettings::LoadFromYAML + AssetRegistry/MaterialManager (mainOffline.cpp:142-198):
 * reads data_dir/settings/global_settings.yaml, assets/{materials,blocks}.yaml */
int vxpt_load_settings(vxpt_ctx *ctx);
/* SceneConfigParser::LoadFromFile (SceneConfig.cpp:6-) -> camera */
int vxpt_load_scene_camera(vxpt_ctx *ctx, const char *scene_yaml, vxpt_camera *out);

/* VoxelEngine::init -> initVoxelsMultiChunk (VoxelSceneGen.cu:341-388): Perlin terrain.
 * height_scale = 32 and freq_den = 32*chunks_x reproduce the reference.  flags:
 * VXPT_TERRAIN_SHADER_BALLS keeps the 10 instanced shader balls (their mesh is missing, so
 * parity scenes drop them); VXPT_TERRAIN_GLOBAL_Y compares world y instead of the chunk-local
 * y the reference uses (the reference repeats the terrain in every chunk layer; identical
 * when chunks_y == 1) -- used for the synthetic 256^3 benchmark world. */
#define VXPT_TERRAIN_SHADER_BALLS 1
#define VXPT_TERRAIN_GLOBAL_Y 2
int vxpt_generate_terrain(vxpt_ctx *ctx, int chunks_x, int chunks_y, int chunks_z, float height_scale,
                          float freq_den, int flags);
/* upload an explicit grid: chunk-major, 32^3 per chunk, x + 32*(z + 32*y) (VoxelChunk.h:12-55) */
int vxpt_upload_voxels(vxpt_ctx *ctx, const uint8_t *ids, int chunks_x, int chunks_y, int chunks_z);
/* MaterialManager GPU table (MaterialManager.cpp:60-170) for block ids 1..12 */
int vxpt_upload_materials(vxpt_ctx *ctx, const vxpt_material *mats, int n_block_ids);
/* SkyModel::update (Sky.cu:355-396): sky + sun maps on the GPU, alias tables on the host */
int vxpt_set_sky(vxpt_ctx *ctx, float time_of_day, float sun_axis_angle_deg, float sun_axis_rotate_deg,
                 float brightness);
/* RenderCamera camera/historyCamera (mainOffline.cpp:227-251) */
int vxpt_set_camera(vxpt_ctx *ctx, const vxpt_camera *cur, const vxpt_camera *prev);
/* Camera matrices as the kernels see them: pos3 dir3 uvToWorld9 worldToUv9 res2 invRes2 tanHalfFov2 yaw pitch */
int vxpt_get_camera(vxpt_ctx *ctx, int which, float out32[32]);
/* Camera::update from yaw/pitch (Camera.h:44-100) after historyCamera = camera (mainOffline.cpp:278-307,
 * the circular-removal test's orientation changes); out32[30..31] of vxpt_get_camera are yaw, pitch */
int vxpt_set_camera_angles(vxpt_ctx *ctx, const float pos[3], float yaw, float pitch, float fov_deg);

/* ---- textures (TextureManager.cu:133-330; shading closesthit.cu:167-254) ---- */
/* load every texture the cube materials name (paths from assets/materials.yaml, relative to root;
 * NULL = data_dir) as RGBA8 mip chains and turn textured shading on; missing or non-square files
 * are skipped (their materials stay untextured).  *loaded = textures loaded */
int vxpt_load_textures(vxpt_ctx *ctx, const char *root, int *loaded);
/* textured shading on/off once loaded (the untextured parity scenes use off) */
int vxpt_enable_textures(vxpt_ctx *ctx, int on);
/* texture table: per texture size, maxLod, maxLod + 1 level offsets in texels (parity hook) */
int vxpt_texture_table(vxpt_ctx *ctx, int32_t *out, int cap, int *n_textures, int64_t *n_texels);

/* ---- instanced block meshes + emissive triangle lights ---- */
/* BlockManager / ModelManager / VoxelEngine::{collectInstanceTransforms, generateInstanceLights}
 * (BlockManager.cpp:7-160, ModelManager.cpp:172-226, ObjUtils.cpp:13-120, VoxelEngine.cu:53-192,
 * 323-520): read blocks 13..29 from assets/blocks.yaml, their models from assets/models.yaml and
 * the OBJ files under root (NULL = data_dir; a missing file leaves the block with no triangles),
 * collect the instances of the current world and build the light table + its alias table.  Both
 * are rebuilt by every later world upload and by edits that place or remove an instanced block.
 * *loaded = block types whose mesh loaded.  The DDA still treats instanced cells as empty. */
int vxpt_load_models(vxpt_ctx *ctx, const char *root, int *loaded);
/* a block type's mesh as loaded: 9 floats (3 corners) and 6 floats (3 texcoords) per triangle */
int vxpt_get_model(vxpt_ctx *ctx, int block_id, float *pos, float *uv, int cap_triangles, int *n_triangles);
/* instances, 5 x int32 each: object id (= block - 1), instance id, cell x, y, z; ordered by object,
 * then instance id (Scene::geometryInstanceIdMap) */
int vxpt_get_instances(vxpt_ctx *ctx, int32_t *out, int cap, int *n_instances);
/* light table summary: per emissive instance (instance id, first light, triangles)
 * (Scene::instanceLightMapping), the light count and the weights' sum
 * (accumulatedLocalLightLuminance); the records are VXPT_BUF_LIGHTS / VXPT_BUF_LIGHT_ALIAS */
int vxpt_get_lights(vxpt_ctx *ctx, uint32_t *mapping, int cap, int *n_mapped, uint32_t *n_lights,
                    float *local_luminance);
/* the last light update's previous -> current light index table (VoxelEngine::buildLightIdMapping /
 * buildIncrementalLightMapping, VoxelEngine.cu:503-633; -1 = the light is gone), its length (the
 * light count before the update, Scene::m_prevNumLights) and whether the next trace pass still
 * applies it to the previous reservoirs (Scene::m_lightsJustUpdated, Restir.h:48-79) */
int vxpt_get_light_remap(vxpt_ctx *ctx, int32_t *remap, int cap, int *prev_num_lights, int *pending);
/* closest hit against the instanced meshes (the IAS the reference's rays traverse besides the
 * voxel faces; meshes.hip): n rays of 8 floats (origin, tmin, direction, tmax); out 4 floats per ray
 * (t, u, v barycentrics, hit 0/1), ids 2 int32 (instance row of vxpt_get_instances, triangle);
 * cull = 1 skips back faces (radiance rays), 0 not (visibility rays).  Ties: smaller t, then row,
 * then triangle.  Parity hook: the path kernels do not consult the meshes yet */
int vxpt_mesh_probe(vxpt_ctx *ctx, const float *rays, int n, int cull, float *out, int32_t *ids);
/* the visibility-ray form of the same query (optixTraverse with OPTIX_RAY_FLAG_DISABLE_CLOSESTHIT,
 * no culling, closesthit.cu:616-625 / 752 / 808): occluded[i] = 1 iff some instanced-mesh
 * triangle, either face, lies in [tmin, tmax] of ray i; the walk stops at the first one */
int vxpt_mesh_occluded(vxpt_ctx *ctx, const float *rays, int n, uint8_t *occluded);
/* the mesh BVH builder on its own (no context, no GPU; test hook): n boxes of 6 floats (lo xyz,
 * hi xyz), leaves of at most leaf_max primitives -> the deepest leaf's depth (<= 40: the walk's
 * stack bound) and the node count; VXPT_ERR_STATE if the depth limit cannot be kept */
int vxpt_bvh_depth(const float *boxes, int n, int leaf_max, int *max_depth, int *n_nodes);

/* ---- voxel edits (VoxelEngine::update click path, VoxelEngine.cu:855-975, 1040-1346) ---- */
/* performRayTraversal (:1040-1166) of the current camera ray on the world.  out: hit, hit x, y, z,
 * hit id, has space to place, place x, y, z, cells walked */
int vxpt_pick_block(vxpt_ctx *ctx, int32_t out[10]);
/* setVoxelAtGlobal + the geometry update (:265-276; VoxelSceneGen.cu:643-786): one cell's id, with
 * the traversal structures updated incrementally; the next trace pass's ReSTIR temporal visibility
 * sees no previous scene (OptixRenderer.cpp:916-919) */
int vxpt_set_block(vxpt_ctx *ctx, int x, int y, int z, int block_id);
/* the click (:906-975): block_id 0 deletes the picked block, another id is placed in front of it;
 * out (may be NULL) = the pick */
int vxpt_click_block(vxpt_ctx *ctx, int block_id, int32_t out[10]);
/* WorldSceneManager::SaveScene / LoadScene (WorldSceneManager.cpp:240-458): chunk files named by
 * the FNV-1a 64 hash of their bytes + a scene yaml with the camera, chunk_config and chunk records;
 * load fills cam_out (may be NULL) and rebuilds the world */
int vxpt_save_world(vxpt_ctx *ctx, const char *scene_yaml, const char *chunk_dir);
int vxpt_load_world(vxpt_ctx *ctx, const char *scene_yaml, const char *chunk_dir, vxpt_camera *cam_out);

/* OptixRenderer::render (OptixRenderer.cpp:411-485): one 1-spp trace pass with the given
 * iterationIndex.  flags: VXPT_TRACE_PRIMARY_ONLY = C2 bring-up mode (DDA + sky + G-buffer). */
#define VXPT_TRACE_PRIMARY_ONLY 1u
/* spp > 1 passes of one frame (OfflineBackend::renderFrame via vxpt_render_frame does this
 * itself): ACCUMULATE adds radiance/spp into the denoiser input, ACCUM_FIRST starts the sum,
 * bits 8..15 carry spp */
#define VXPT_TRACE_ACCUMULATE 2u
#define VXPT_TRACE_ACCUM_FIRST 4u
#define VXPT_TRACE_SPP(n) ((uint32_t)(n) << 8)
int vxpt_trace(vxpt_ctx *ctx, int32_t iteration_index, uint32_t flags);
/* Denoiser::run (Denoiser.cu:24-408); iteration_index = value after render() incremented it */
int vxpt_denoise(vxpt_ctx *ctx, const vxpt_denoise_params *p, int32_t frame_num, int32_t iteration_index);
/* one denoiser pass on the current buffers, over the context's band (multi-GPU schedule,
 * parity hooks): 0 firefly (arg = reservoir parity), 2 temporal accumulation, 3 history fix,
 * 4 history clamping, 5 a-trous smem, 6 a-trous ping->pong (arg step, arg2 frame index),
 * 7 a-trous pong->ping, 10 final a-trous ping->pong + output, 11 world positions (band +/- 40
 * rows; needed before 0, 3, 5, 6, 7, 10), 12 frame-0 history init, 13 output copy (arg: source
 * 0 illum, 1 ping, 2 pong, 3 prev illum), 14 history copies */
int vxpt_denoise_pass(vxpt_ctx *ctx, const vxpt_denoise_params *p, int pass, int arg, int arg2);
/* OfflineBackend::renderFrame: spp trace passes (radiance averaged) + denoise.  frame_num as
 * OfflineBackend::m_frameNum; iteration indices frame_num*spp .. +spp-1. */
int vxpt_render_frame(vxpt_ctx *ctx, const vxpt_denoise_params *p, int32_t frame_num, int32_t spp);
/* n_frames consecutive vxpt_render_frame calls (frames frame0 .. frame0+n_frames-1) with the
 * camera, world and lights left as they are: mainOffline's frame loop for a static camera.  The
 * buffers afterwards equal those calls' bit for bit; each frame's first trace pass is enqueued
 * beside the previous frame's last one, so the sequence takes less time (banded contexts too); the
 * host waits for each denoiser chain before it enqueues the next frame's later passes, so the call
 * returns only after the last frame's chain has been enqueued and the others have run.  Timing (HIP events):
 * frame_ms is the mean per frame, denoise_ms the mean of the frames' denoiser chains (each timed on
 * its own; they run alone), trace_ms the mean per frame without them. */
int vxpt_render_frames(vxpt_ctx *ctx, const vxpt_denoise_params *p, int32_t frame0, int32_t n_frames,
                       int32_t spp);
/* the denoiser parameters of global_settings.yaml's `denoising` section (GlobalSettings.h:82-141),
 * the ones every call above uses when p = NULL */
int vxpt_get_denoise_params(vxpt_ctx *ctx, vxpt_denoise_params *out);

/* PostProcessor::run (PostProcessor.cu:74-122): histogram auto-exposure, bloom, lens flare,
 * vignette, filmic tone mapping, crosshair; the denoiser output -> VXPT_BUF_FRAME.  p = NULL
 * takes the yaml values (vxpt_load_settings); dt_ms = Timer::getDeltaTime (milliseconds) for the
 * exposure adaptation (OfflineBackend.cpp:79; any dt >= 1 ms adapts fully in one frame). */
int vxpt_get_post_params(vxpt_ctx *ctx, vxpt_post_params *out);
/* the lens flare's sun (ProjectSunToScreen, PostProcessingPipeline.cu:187-206): on-screen flag,
 * pixel x, y, uv, and the accumulated sun luminance (parity hook) */
int vxpt_get_sun_projection(vxpt_ctx *ctx, float out6[6]);
int vxpt_postprocess(vxpt_ctx *ctx, const vxpt_post_params *p, float dt_ms);
/* vxpt_postprocess over the bands of vxpt_band_link'ed contexts of one process (the 1-GPU stand-in
 * for the RCCL band path, which vxpt_postprocess takes by itself on a context with a communicator):
 * the denoiser output's 1-row halo, the histogram summed over the bands, the bloom's halo */
int vxpt_postprocess_linked(vxpt_ctx **ctxs, int n, const vxpt_post_params *p, float dt_ms);
/* OfflineBackend::writeFrameBufferToPNG (OfflineBackend.cpp:191-221): rgba = W*H float4 (the
 * frame), clamped to [0,1], x255 truncated, rows flipped, written as 8-bit RGB PNG */
int vxpt_write_png_rgba32f(const char *path, int w, int h, const float *rgba);
/* 8-bit PNG reader (query with pixels = NULL, then read w*h*channels bytes) */
int vxpt_read_png(const char *path, int *w, int *h, int *channels, uint8_t *pixels, size_t cap);
/* ObjUtils::extractMeshFromOBJ (ObjUtils.cpp:13-120), no context: one vertex per face corner,
 * 9 floats (positions) and 6 floats (texcoords) per triangle; *n_triangles = the file's count,
 * at most cap_triangles written.  VXPT_ERR_IO when the file is missing or a face corner is bad */
int vxpt_read_obj(const char *path, float *pos, float *uv, int cap_triangles, int *n_triangles);
/* ImageDiff::compare / generateDiffImage (renderer/util/ImageDiff.cpp:94-185): the canonical-image
 * gate of mainOffline --test-canonical (mainOffline.cpp:450-497) */
int vxpt_image_diff(const char *png_a, const char *png_b, vxpt_image_diff_result *out);
int vxpt_image_diff_png(const char *png_a, const char *png_b, const char *diff_png);

/* multi-GPU band partition: the context traces and denoises only rows
 * [row_begin, row_end) (8-aligned; 0,0 = whole frame) of full-frame buffers.  Rows
 * outside the band are filled by the host from the neighbours' bands with
 * vxpt_copy_rows (the transport -- RCCL over xGMI -- belongs to the host process). */
int vxpt_set_band(vxpt_ctx *ctx, int row_begin, int row_end);
/* bytes per row of a per-pixel buffer (negative if it has no row layout) */
int vxpt_row_bytes(vxpt_ctx *ctx, int which);
/* copy `rows` rows starting at row y between a buffer and device memory `dev`
 * (to_buffer = 1: dev -> buffer), enqueued on the context stream */
int vxpt_copy_rows(vxpt_ctx *ctx, int which, int y, int rows, void *dev, int to_buffer);
/* one halo exchange of the band schedule below, for a host-driven schedule over the context's RCCL
 * communicator: the buffers of buffer_mask (bit b = buffer id b < 32, per-pixel buffers only),
 * `rows` rows with each band neighbour (vxpt_halo_plan), grouped ncclSend/ncclRecv on the context
 * stream.  A no-op for one band; VXPT_ERR_STATE without a communicator. */
int vxpt_exchange_halo(vxpt_ctx *ctx, uint32_t buffer_mask, int rows);
/* the band partition's pure functions (no context, no GPU): rows [row_begin, row_end) of `rank`
 * (8-aligned equal bands, the last takes the rest), and the halo plan of a `rows`-deep exchange:
 * up to 2 entries of 5 int32 (peer, send row, send rows, receive row, receive rows) for the
 * neighbours rank -/+ 1, both sides of a border moving min(rows, the two band heights) rows */
int vxpt_band_rows(int height, int nranks, int rank, int *row_begin, int *row_end);
int vxpt_halo_plan(int height, int nranks, int rank, int rows, int32_t out[10], int *n_entries);
/* halo depths a banded frame exchanges for a camera that turned from prev to cur between passes:
 * trace_rows (ReSTIR temporal taps: 64 rows around the reprojected row, >= 72) and history_rows
 * (the temporal accumulation's bicubic history taps, >= 2).  VXPT_ERR_STATE when the camera
 * translated (depth-dependent parallax: see vxpt_band_halo_rows_near), part of a band falls behind
 * the previous camera, or the trace halo is deeper than a band: vxpt_render_frame / _linked refuse
 * such a frame the same way. */
int vxpt_band_halo_rows(const vxpt_camera *cur, const vxpt_camera *prev, int width, int height, int nranks,
                        int *trace_rows, int *history_rows);
/* the same for a camera that may also translate: near_depth > 0 bounds every primary hit's distance
 * from the camera (a pixel's reprojected row is monotone in its hit distance, so the rows at
 * near_depth and at infinity bound it).  vxpt_render_frame / _linked use the world's own bound,
 * vxpt_nearest_surface: the distance from pos to the nearest non-air cell grown by one cell, or by
 * the loaded meshes' largest overhang past their cell when that is more (vxpt_load_models), searched
 * up to 64 cells (host mirror of the world; no GPU work). */
int vxpt_band_halo_rows_near(const vxpt_camera *cur, const vxpt_camera *prev, int width, int height, int nranks,
                             float near_depth, int *trace_rows, int *history_rows);
int vxpt_nearest_surface(vxpt_ctx *ctx, const float pos[3], float *dist);
/* end-of-frame gather: every band's rows of a per-pixel buffer (e.g. VXPT_BUF_OUTPUT, or
 * VXPT_BUF_FRAME after vxpt_postprocess) into the root rank's buffer, which then holds the whole
 * frame (RCCL: ncclSend to the root, ncclRecv per band at the root; blocking) */
int vxpt_band_gather(vxpt_ctx *ctx, int which, int root);
int vxpt_band_gather_linked(vxpt_ctx **ctxs, int n, int which, int root);

/* Multi-GPU band partition driven by the library (replaces the single-GPU
 * OfflineBackend::renderFrame, OfflineBackend.cpp:46-89, with one band per GPU).  One process
 * per GPU: rank 0 calls vxpt_band_comm_id (an RCCL unique id, 128 bytes), the host broadcasts
 * it, every rank calls vxpt_band_comm_init.  The context then owns rows band_rows(H, nranks,
 * rank) and vxpt_render_frame renders that band, enqueueing every halo exchange (grouped
 * ncclSend/ncclRecv with the neighbours rank +/- 1, rows moved in place) on the context
 * stream.  Bands must be >= 72 rows tall; a camera that turns between frames deepens the
 * halos (vxpt_band_halo_rows). */
int vxpt_band_comm_id(void *id, size_t bytes);
int vxpt_band_comm_init(vxpt_ctx *ctx, const void *id, size_t bytes, int nranks, int rank);
/* the same with an uneven partition: band r = rows [row_splits[r], row_splits[r + 1]) of nranks + 1
 * boundaries (0 first, height last, inner ones 8-aligned, every band >= 72 rows), the same array on
 * every rank; NULL = the equal bands.  vxpt_band_balance proposes one from measured band times. */
int vxpt_band_comm_init_rows(vxpt_ctx *ctx, const void *id, size_t bytes, int nranks, int rank,
                             const int32_t *row_splits);
/* The same schedule over n contexts of one process (tests, one-GPU boxes): context k owns band
 * k of n; halo rows move by device copies between the contexts. */
int vxpt_band_link(vxpt_ctx **ctxs, int n);
int vxpt_band_link_rows(vxpt_ctx **ctxs, int n, const int32_t *row_splits);
/* cost-balanced boundaries (pure host function): band_ms[r] = the measured time of band r of the
 * partition row_splits; block_cost = the frame's cost per 8-row block (ceil(height / 8) floats, kept
 * by the caller between calls; first entry < 0 = no estimate yet) is refined with them -- each band's
 * blocks scaled to sum to its time -- and out_splits (nranks + 1) cut the cumulative cost into equal
 * parts on block boundaries, every band >= 72 rows.  Screen rows cost unevenly (a band that sees
 * the horizon walks far more cells than one that sees the ground under the camera), so equal bands
 * leave the slowest rank well above the mean. */
int vxpt_band_balance(int height, int nranks, const int32_t *row_splits, const float *band_ms, float *block_cost,
                      int32_t *out_splits);
int vxpt_render_frame_linked(vxpt_ctx **ctxs, int n, const vxpt_denoise_params *p, int32_t frame_num,
                             int32_t spp);
/* n_frames banded frames over linked contexts with the RCCL run's own pipelined schedule (a banded
 * vxpt_render_frames: the next frame's first pass-halves enqueued beside the last second half and its
 * exchange, the denoiser chain after them, the later first halves gated on the host behind the chain),
 * device copies as the transport; results equal n_frames vxpt_render_frame_linked calls bit for bit. */
int vxpt_render_frames_linked(vxpt_ctx **ctxs, int n, const vxpt_denoise_params *p, int32_t frame0,
                              int32_t n_frames, int32_t spp);

/* Halo-exchange instrumentation of a banded context (no reference counterpart; the first multi-GPU
 * run explains itself with it).  With collection on, every exchange group of a banded
 * vxpt_render_frame(s) / vxpt_render_frame_linked is bracketed by HIP events on the stream it runs on
 * (ordered groups on the context stream, overlapped ones on the exchange stream beside the next pass)
 * and its bytes are counted per neighbour, and each banded frame's trace span (its passes with their
 * exchanges) and denoiser span are timed.  Totals since the last enable; vxpt_band_stats syncs the
 * context's streams first.  (vxpt_timings of a banded vxpt_render_frames run holds the last frame's
 * trace / denoiser split and the run's mean frame time; these spans are every frame's.) */
typedef struct vxpt_band_stat {
    int32_t frames;            /* banded frames rendered while collecting */
    int32_t groups;            /* exchange groups: one RCCL group, or one context's set of linked copies */
    int32_t groups_ordered;    /* of them, on the context stream (in stream order with the kernels) */
    float exchange_ms;         /* HIP-event time inside the ordered groups, summed */
    float exchange_overlap_ms; /* the same for the overlapped groups (exchange stream) */
    float trace_ms;            /* the frames' trace spans, summed */
    float denoise_ms;          /* the frames' denoiser spans, summed */
    double bytes_up;           /* bytes sent to the band above (rank - 1) */
    double bytes_down;         /* bytes sent to the band below (rank + 1) */
    int32_t row_begin, row_end;
} vxpt_band_stat;
/* on != 0: collection on, totals reset; 0: off */
int vxpt_band_stats_enable(vxpt_ctx *ctx, int on);
int vxpt_band_stats(vxpt_ctx *ctx, vxpt_band_stat *out);

/* on != 0: the history clamp records its decisions in VXPT_BUF_CLAMP_DECISION (parity hook; one more
 * plane store per pixel while on) */
int vxpt_debug_clamp_decisions(vxpt_ctx *ctx, int on);

/* copy any logical buffer to/from host memory (parity hooks, PNG output).  Uploads of G-buffer planes
 * mark the slots' ReSTIR tap records stale; the next trace rebuilds them from NORMAL_ROUGH, ALBEDO,
 * MAT_PARAM.x and DEPTH (k_pack_rec).  The taps take their geometric normal from NORMAL_ROUGH: the trace
 * writes the same normal to both planes, so an uploaded GEO_NORMAL_THIN that differs from
 * NORMAL_ROUGH.xyz is not seen by the temporal taps (GetPrevSurface, Restir.h:359-378, reads it).  In a
 * banded context such an upload must also cover the trace halo rows (the library's own exchanges move
 * the records, not the planes, between passes). */
int vxpt_readback(vxpt_ctx *ctx, int which, void *host, size_t bytes);
int vxpt_upload(vxpt_ctx *ctx, int which, const void *host, size_t bytes);
/* sky alias table (Vose, AliasTable.cu:66-153): q,p floats and alias ints, 1024*512 each */
int vxpt_get_sky_alias(vxpt_ctx *ctx, float *q, float *p, int32_t *alias, float sun_dir[3]);
int vxpt_timings(vxpt_ctx *ctx, vxpt_timing *out);
int vxpt_sync(vxpt_ctx *ctx);
/* raw stream handle (hipStream_t) for hosts that enqueue their own work */
void *vxpt_stream(vxpt_ctx *ctx);
/* DDA probe: n rays (o3 d3 tmin tmax) -> n x (hit x y z face id) + t; mode 0 closest, 2 occluded;
 * mode | 4: the same walks handed over through the straggler save/resume state after every iteration */
int vxpt_probe_rays(vxpt_ctx *ctx, int n, const float *rays, int32_t *out6, float *t, int mode);
/* blue-noise sampler probe: n queries (pixel x, pixel y, iterationIndex, dimension) ->
 * BlueNoiseRandGenerator::rand (RandGen.h:21-45) as the trace kernel evaluates it */
int vxpt_probe_rng(vxpt_ctx *ctx, int n, const int32_t *q4, float *out);
/* ray-queue counters of the last trace pass (no reference counterpart: the wavefront's
 * own instrumentation, read after the pass): for each of the 16 queues q (4*segment + kind,
 * kind 1 BRDF-candidate closest-hit rays, 2 NEE visibility rays, 3 ReSTIR visibility rays)
 * out[3q] = rays queued, out[3q+1] = walks deferred to the straggler queue (level 1),
 * out[3q+2] = walks deferred again (level 2).  cap >= 48 */
int vxpt_trace_counters(vxpt_ctx *ctx, uint32_t *out, int cap);

#ifdef __cplusplus
}
#endif
#endif /* VXPT_H */
