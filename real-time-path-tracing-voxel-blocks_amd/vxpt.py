"""vxpt -- Python host mirror of the reference's offline render interface.

The product is libvxpt.so (HIP kernels for gfx950 + C++ host runtime, C ABI in
include/vxpt.h).  This module only binds that ABI with ctypes and mirrors the
reference's OfflineBackend / mainOffline call order
(renderer/core/OfflineBackend.cpp:46-89, mainOffline.cpp:142-251) so host
programs and tests read like the reference's own driver.  It never computes
pixels itself: if libvxpt.so is missing or cannot reach a GPU every entry
point raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("VXPT_LIB") or os.path.join(_HERE, "libvxpt.so")
DATA_DIR = os.path.join(REPO, "data")

# logical buffers (include/vxpt.h enum vxpt_buffer)
BUF = dict(ILLUM=0, DEPTH=1, NORMAL_ROUGH=2, GEO_NORMAL_THIN=3, ALBEDO=4, MATERIAL=5, MAT_PARAM=6, MOTION=7,
           PREV_NORMAL_ROUGH=8, PREV_GEO_NORMAL_THIN=9, PREV_ALBEDO=10, PREV_MAT_PARAM=11, PREV_DEPTH=12,
           PREV_MATERIAL=13, RESERVOIRS=14, PING=15, PONG=16, PREV_ILLUM=17, PREV_FAST=18, HIST_LEN=19,
           PREV_HIST_LEN=20, OUTPUT=21, SKY=32, SUN=33, VOXELS=34, RES_EVEN=35, RES_ODD=36, WPOS=37, FRAME=38,
           OCTANT_TABLES=39, CELL_MASKS=40, BRICK_IDS=41, MACRO_MASKS=42, TEXELS=43, LIGHTS=44,
           LIGHT_ALIAS=45, BLOOM=46, TAP_RECORD=47, BOX_TABLES=48, CLAMP_DECISION=49)
FLOAT1_BUFS = {1, 5, 12, 13, 19, 20, 49}
RESERVOIR_DTYPE = np.dtype([("lightData", "<u4"), ("uvData", "<u4"), ("weightSum", "<f4"), ("targetPdf", "<f4"),
                            ("M", "<f4")])
ALIAS_DTYPE = np.dtype([("q", "<f4"), ("p", "<f4"), ("alias", "<i4")])
TRACE_PRIMARY_ONLY = 1


class VxptError(RuntimeError):
    pass


class Config(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("device", ctypes.c_int32),
                ("row_begin", ctypes.c_int32), ("row_end", ctypes.c_int32),
                ("total_bounce_limit", ctypes.c_int32), ("diffuse_bounce_limit", ctypes.c_int32),
                ("data_dir", ctypes.c_char_p)]


class Camera(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_float * 3), ("dir", ctypes.c_float * 3), ("fov_deg", ctypes.c_float)]


class Material(ctypes.Structure):
    _fields_ = [("albedo", ctypes.c_float * 3), ("roughness", ctypes.c_float), ("translucency", ctypes.c_float),
                ("metallic", ctypes.c_int32), ("material_id", ctypes.c_int32), ("thinfilm", ctypes.c_int32)]


class DenoiseParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in (
        "max_accumulated_frame_num", "max_fast_accumulated_frame_num", "phi_luminance", "lobe_angle_fraction",
        "roughness_fraction", "depth_threshold", "disocclusion_threshold", "disocclusion_threshold_alternate",
        "denoising_range")] + [(n, ctypes.c_int32) for n in (
            "enable_temporal_accumulation", "enable_history_fix", "enable_history_clamping",
            "enable_spatial_filtering", "enable_firefly_filter", "atrous_iteration_num")]

    @classmethod
    def defaults(cls):
        """global_settings.yaml denoising section (atrousIterationNum: 1)."""
        return cls(30.0, 6.0, 2.0, 0.5, 0.15, 0.003, 0.01, 0.05, 500000.0, 1, 1, 1, 1, 1, 1)


class PostParams(ctypes.Structure):
    """vxpt_post_params (ToneMappingParams + PostProcessingPipelineParams, GlobalSettings.h:10-186)."""
    _fields_ = [("manual_exposure", ctypes.c_float), ("tone_mapping_curve", ctypes.c_int32)] + \
        [(n, ctypes.c_float) for n in ("white_point", "contrast", "saturation", "lift", "gain")] + \
        [("enable_bloom", ctypes.c_int32)] + \
        [(n, ctypes.c_float) for n in ("bloom_threshold", "bloom_intensity", "bloom_radius")] + \
        [("enable_auto_exposure", ctypes.c_int32)] + \
        [(n, ctypes.c_float) for n in ("exposure_speed", "exposure_min", "exposure_max", "exposure_compensation",
                                       "histogram_min_percent", "histogram_max_percent", "target_luminance")] + \
        [("enable_vignette", ctypes.c_int32)] + \
        [(n, ctypes.c_float) for n in ("vignette_strength", "vignette_radius", "vignette_smoothness")] + \
        [("enable_lens_flare", ctypes.c_int32)] + \
        [(n, ctypes.c_float) for n in ("lens_flare_intensity", "lens_flare_ghost_spacing")] + \
        [("lens_flare_ghost_count", ctypes.c_int32)] + \
        [(n, ctypes.c_float) for n in ("lens_flare_halo_radius", "lens_flare_sun_size", "lens_flare_distortion")] + \
        [("draw_crosshair", ctypes.c_int32)]


class ImageDiffResult(ctypes.Structure):
    _fields_ = [("total_pixels", ctypes.c_int32), ("different_pixels", ctypes.c_int32),
                ("pixel_difference_ratio", ctypes.c_float), ("rmse", ctypes.c_float), ("ssim", ctypes.c_float),
                ("is_identical", ctypes.c_int32), ("is_very_close", ctypes.c_int32), ("is_close", ctypes.c_int32)]


TUNING_FIELDS = ("dda_boxes", "box_cap", "box_cap_up", "brick_steps", "cam_steps", "iter_cap", "iter_cap2",
                 "resume_wg_per_cu", "sort_mode", "overlap", "state_sets", "firefly_fused", "ta_supertiles",
                 "hf_split", "stencil_tile", "front_streams", "lds_bricks", "resume_split", "later_split",
                 "restir_waves", "ghost_rows", "chain_gate", "sky_exit", "xcd_order", "iter_cap3", "iter_cap4")


class Tuning(ctypes.Structure):
    """vxpt_tuning: the context's schedule (no field changes a result)."""
    _fields_ = [(n, ctypes.c_int32) for n in TUNING_FIELDS]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n in TUNING_FIELDS}


class Timing(ctypes.Structure):
    _fields_ = [("trace_ms", ctypes.c_float), ("denoise_ms", ctypes.c_float), ("sky_ms", ctypes.c_float),
                ("frame_ms", ctypes.c_float), ("host_ms", ctypes.c_float)]


class BandStat(ctypes.Structure):  # vxpt_band_stat
    _fields_ = [("frames", ctypes.c_int32), ("groups", ctypes.c_int32), ("groups_ordered", ctypes.c_int32),
                ("exchange_ms", ctypes.c_float), ("exchange_overlap_ms", ctypes.c_float),
                ("trace_ms", ctypes.c_float), ("denoise_ms", ctypes.c_float),
                ("bytes_up", ctypes.c_double), ("bytes_down", ctypes.c_double),
                ("row_begin", ctypes.c_int32), ("row_end", ctypes.c_int32)]


_lib = None


def load_library(path=LIB_PATH):
    """Load libvxpt.so; raises (no fallback) when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise VxptError("libvxpt.so not built (%s); run __graft_entry__.build()" % path)
    lib = ctypes.CDLL(path)
    P, I, F, U32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_uint32
    sigs = {
        "vxpt_create": (I, [ctypes.POINTER(Config), ctypes.POINTER(P)]),
        "vxpt_destroy": (None, [P]),
        "vxpt_last_error": (ctypes.c_char_p, [P]),
        "vxpt_load_settings": (I, [P]),
        "vxpt_load_scene_camera": (I, [P, ctypes.c_char_p, ctypes.POINTER(Camera)]),
        "vxpt_generate_terrain": (I, [P, I, I, I, F, F, I]),
        "vxpt_upload_voxels": (I, [P, P, I, I, I]),
        "vxpt_upload_materials": (I, [P, ctypes.POINTER(Material), I]),
        "vxpt_set_sky": (I, [P, F, F, F, F]),
        "vxpt_set_camera": (I, [P, ctypes.POINTER(Camera), ctypes.POINTER(Camera)]),
        "vxpt_get_camera": (I, [P, I, P]),
        "vxpt_set_camera_angles": (I, [P, P, F, F, F]),
        "vxpt_pick_block": (I, [P, P]),
        "vxpt_load_textures": (I, [P, ctypes.c_char_p, P]),
        "vxpt_enable_textures": (I, [P, I]),
        "vxpt_texture_table": (I, [P, P, I, P, P]),
        "vxpt_load_models": (I, [P, ctypes.c_char_p, P]),
        "vxpt_read_obj": (I, [ctypes.c_char_p, P, P, I, P]),
        "vxpt_get_model": (I, [P, I, P, P, I, P]),
        "vxpt_get_instances": (I, [P, P, I, P]),
        "vxpt_get_lights": (I, [P, P, I, P, P, P]),
        "vxpt_get_light_remap": (I, [P, P, I, P, P]),
        "vxpt_mesh_probe": (I, [P, P, I, I, P, P]),
        "vxpt_mesh_occluded": (I, [P, P, I, P]),
        "vxpt_set_block": (I, [P, I, I, I, I]),
        "vxpt_click_block": (I, [P, I, P]),
        "vxpt_save_world": (I, [P, ctypes.c_char_p, ctypes.c_char_p]),
        "vxpt_load_world": (I, [P, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Camera)]),
        "vxpt_trace": (I, [P, ctypes.c_int32, U32]),
        "vxpt_denoise": (I, [P, ctypes.POINTER(DenoiseParams), ctypes.c_int32, ctypes.c_int32]),
        "vxpt_denoise_pass": (I, [P, ctypes.POINTER(DenoiseParams), I, I, I]),
        "vxpt_render_frame": (I, [P, ctypes.POINTER(DenoiseParams), ctypes.c_int32, ctypes.c_int32]),
        "vxpt_render_frames": (I, [P, ctypes.POINTER(DenoiseParams), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
        "vxpt_exchange_halo": (I, [P, U32, I]),
        "vxpt_readback": (I, [P, I, P, ctypes.c_size_t]),
        "vxpt_upload": (I, [P, I, P, ctypes.c_size_t]),
        "vxpt_get_sky_alias": (I, [P, P, P, P, P]),
        "vxpt_timings": (I, [P, ctypes.POINTER(Timing)]),
        "vxpt_band_stats_enable": (I, [P, I]),
        "vxpt_debug_clamp_decisions": (I, [P, I]),
        "vxpt_band_stats": (I, [P, ctypes.POINTER(BandStat)]),
        "vxpt_tuning_defaults": (I, [ctypes.POINTER(Tuning)]),
        "vxpt_get_tuning": (I, [P, ctypes.POINTER(Tuning)]),
        "vxpt_set_tuning": (I, [P, ctypes.POINTER(Tuning)]),
        "vxpt_sync": (I, [P]),
        "vxpt_stream": (P, [P]),
        "vxpt_probe_rays": (I, [P, I, P, P, P, I]),
        "vxpt_probe_rng": (I, [P, I, P, P]),
        "vxpt_trace_counters": (I, [P, P, I]),
        "vxpt_set_band": (I, [P, I, I]),
        "vxpt_row_bytes": (I, [P, I]),
        "vxpt_copy_rows": (I, [P, I, I, I, P, I]),
        "vxpt_get_post_params": (I, [P, ctypes.POINTER(PostParams)]),
        "vxpt_postprocess": (I, [P, ctypes.POINTER(PostParams), F]),
        "vxpt_postprocess_linked": (I, [ctypes.POINTER(P), I, ctypes.POINTER(PostParams), F]),
        "vxpt_get_sun_projection": (I, [P, P]),
        "vxpt_get_denoise_params": (I, [P, ctypes.POINTER(DenoiseParams)]),
        "vxpt_write_png_rgba32f": (I, [ctypes.c_char_p, I, I, P]),
        "vxpt_read_png": (I, [ctypes.c_char_p, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(I), P,
                              ctypes.c_size_t]),
        "vxpt_image_diff": (I, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ImageDiffResult)]),
        "vxpt_image_diff_png": (I, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]),
        "vxpt_band_comm_id": (I, [P, ctypes.c_size_t]),
        "vxpt_band_comm_init": (I, [P, P, ctypes.c_size_t, I, I]),
        "vxpt_band_link": (I, [ctypes.POINTER(P), I]),
        "vxpt_band_comm_init_rows": (I, [P, P, ctypes.c_size_t, I, I, P]),
        "vxpt_band_link_rows": (I, [ctypes.POINTER(P), I, P]),
        "vxpt_band_balance": (I, [I, I, P, P, P, P]),
        "vxpt_render_frame_linked": (I, [ctypes.POINTER(P), I, ctypes.POINTER(DenoiseParams), ctypes.c_int32,
                                         ctypes.c_int32]),
        "vxpt_render_frames_linked": (I, [ctypes.POINTER(P), I, ctypes.POINTER(DenoiseParams), ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32]),
        "vxpt_band_rows": (I, [I, I, I, ctypes.POINTER(I), ctypes.POINTER(I)]),
        "vxpt_bvh_depth": (I, [P, I, I, ctypes.POINTER(I), ctypes.POINTER(I)]),
        "vxpt_halo_plan": (I, [I, I, I, I, P, ctypes.POINTER(I)]),
        "vxpt_band_halo_rows": (I, [ctypes.POINTER(Camera), ctypes.POINTER(Camera), I, I, I, ctypes.POINTER(I),
                                    ctypes.POINTER(I)]),
        "vxpt_band_halo_rows_near": (I, [ctypes.POINTER(Camera), ctypes.POINTER(Camera), I, I, I, ctypes.c_float,
                                         ctypes.POINTER(I), ctypes.POINTER(I)]),
        "vxpt_nearest_surface": (I, [P, P, ctypes.POINTER(ctypes.c_float)]),
        "vxpt_band_gather": (I, [P, I, I]),
        "vxpt_band_gather_linked": (I, [ctypes.POINTER(P), I, I, I]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


class Renderer:
    """One GPU's share of the offline renderer (OfflineBackend + OptixRenderer +
    Denoiser + SkyModel singletons of the reference, as one context)."""

    def __init__(self, width, height, device=0, rows=None, bounces=(3, 1), data_dir=DATA_DIR):
        self.lib = load_library()
        self.W, self.H = int(width), int(height)
        r0, r1 = rows if rows else (0, 0)
        cfg = Config(self.W, self.H, device, r0, r1, bounces[0], bounces[1], data_dir.encode())
        ctx = ctypes.c_void_p()
        rc = self.lib.vxpt_create(ctypes.byref(cfg), ctypes.byref(ctx))
        self.ctx = ctx
        if rc != 0:
            msg = self.lib.vxpt_last_error(ctx).decode() if ctx.value else ""
            if ctx.value:
                self.lib.vxpt_destroy(ctx)
            self.ctx = None
            raise VxptError("vxpt_create failed (%d) %s" % (rc, msg))

    def _chk(self, rc, what):
        if rc != 0:
            raise VxptError("%s failed (%d): %s" % (what, rc, self.lib.vxpt_last_error(self.ctx).decode()))

    def close(self):
        if self.ctx:
            self.lib.vxpt_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- scene set-up (mainOffline.cpp:142-251) ---
    def nearest_surface(self, pos):
        """vxpt_nearest_surface: a lower bound on the distance from pos to any primary hit (the
        nearest non-air cell grown by one cell, searched up to 64 cells)"""
        d = ctypes.c_float(0.0)
        p = (ctypes.c_float * 3)(*pos)
        self._chk(self.lib.vxpt_nearest_surface(self.ctx, p, ctypes.byref(d)), "vxpt_nearest_surface")
        return d.value

    def load_settings(self):
        self._chk(self.lib.vxpt_load_settings(self.ctx), "vxpt_load_settings")

    def scene_camera(self, path=None):
        cam = Camera()
        self._chk(self.lib.vxpt_load_scene_camera(self.ctx, path.encode() if path else None, ctypes.byref(cam)),
                  "vxpt_load_scene_camera")
        return cam

    def generate_terrain(self, chunks=(2, 1, 2), height_scale=32.0, freq_den=None, keep_shader_balls=False,
                         global_y=False):
        if freq_den is None:
            freq_den = 32.0 * chunks[0]
        flags = (1 if keep_shader_balls else 0) | (2 if global_y else 0)
        self._chk(self.lib.vxpt_generate_terrain(self.ctx, chunks[0], chunks[1], chunks[2], float(height_scale),
                                                 float(freq_den), flags), "vxpt_generate_terrain")
        self.chunks = tuple(chunks)

    def upload_voxels(self, ids, chunks):
        ids = np.ascontiguousarray(ids, dtype=np.uint8)
        self._chk(self.lib.vxpt_upload_voxels(self.ctx, _ptr(ids), chunks[0], chunks[1], chunks[2]),
                  "vxpt_upload_voxels")
        self.chunks = tuple(chunks)

    def set_sky(self, time_of_day=0.25, axis_angle=45.0, axis_rotate=0.0, brightness=1.0):
        self._chk(self.lib.vxpt_set_sky(self.ctx, time_of_day, axis_angle, axis_rotate, brightness), "vxpt_set_sky")

    def set_camera(self, pos, direction, fov=90.0, prev=None):
        cur = Camera((ctypes.c_float * 3)(*pos), (ctypes.c_float * 3)(*direction), fov)
        pv = None
        if prev is not None:
            pv = ctypes.byref(Camera((ctypes.c_float * 3)(*prev[0]), (ctypes.c_float * 3)(*prev[1]), prev[2]))
        self._chk(self.lib.vxpt_set_camera(self.ctx, ctypes.byref(cur), pv), "vxpt_set_camera")

    def camera_info(self, which=0):
        out = np.zeros(32, np.float32)
        self._chk(self.lib.vxpt_get_camera(self.ctx, which, _ptr(out)), "vxpt_get_camera")
        return out

    def set_camera_angles(self, pos, yaw, pitch, fov=90.0):
        """historyCamera = camera, then Camera::update from yaw/pitch (radians)."""
        p = np.ascontiguousarray(pos, np.float32)
        self._chk(self.lib.vxpt_set_camera_angles(self.ctx, _ptr(p), float(yaw), float(pitch), float(fov)),
                  "vxpt_set_camera_angles")

    # --- textures (TextureManager; closesthit.cu:167-254) ---
    def load_textures(self, root=None):
        n = ctypes.c_int(0)
        self._chk(self.lib.vxpt_load_textures(self.ctx, str(root).encode() if root else None, ctypes.byref(n)),
                  "vxpt_load_textures")
        return n.value

    def enable_textures(self, on=True):
        self._chk(self.lib.vxpt_enable_textures(self.ctx, int(bool(on))), "vxpt_enable_textures")

    def texture_table(self):
        """[(size, maxLod, [level offsets in texels])], total texels."""
        n, nt = ctypes.c_int(0), ctypes.c_int64(0)
        self._chk(self.lib.vxpt_texture_table(self.ctx, None, 0, ctypes.byref(n), ctypes.byref(nt)),
                  "vxpt_texture_table")
        out = np.zeros(16 * max(n.value, 1), np.int32)
        self._chk(self.lib.vxpt_texture_table(self.ctx, _ptr(out), len(out), ctypes.byref(n), ctypes.byref(nt)),
                  "vxpt_texture_table")
        tabs, k = [], 0
        for _ in range(n.value):
            size, ml = int(out[k]), int(out[k + 1])
            tabs.append((size, ml, [int(v) for v in out[k + 2:k + 3 + ml]]))
            k += 3 + ml
        self._ntexels = nt.value
        return tabs, nt.value

    # --- instanced meshes + emissive triangle lights ---
    def load_models(self, root=None):
        """blocks 13..29 + models.yaml + the OBJ files under root; returns block types loaded."""
        n = ctypes.c_int(0)
        self._chk(self.lib.vxpt_load_models(self.ctx, str(root).encode() if root else None, ctypes.byref(n)),
                  "vxpt_load_models")
        return n.value

    def model(self, block_id):
        """(pos [T,3,3], uv [T,3,2]) of a block type's loaded mesh."""
        n = ctypes.c_int(0)
        self._chk(self.lib.vxpt_get_model(self.ctx, int(block_id), None, None, 0, ctypes.byref(n)), "vxpt_get_model")
        pos, uv = np.zeros((n.value, 3, 3), np.float32), np.zeros((n.value, 3, 2), np.float32)
        if n.value:
            self._chk(self.lib.vxpt_get_model(self.ctx, int(block_id), _ptr(pos), _ptr(uv), n.value, ctypes.byref(n)),
                      "vxpt_get_model")
        return pos, uv

    def instances(self):
        """int32 [N, 5]: object id, instance id, x, y, z."""
        n = ctypes.c_int(0)
        self._chk(self.lib.vxpt_get_instances(self.ctx, None, 0, ctypes.byref(n)), "vxpt_get_instances")
        out = np.zeros((n.value, 5), np.int32)
        if n.value:
            self._chk(self.lib.vxpt_get_instances(self.ctx, _ptr(out), n.value, ctypes.byref(n)), "vxpt_get_instances")
        return out

    def mesh_probe(self, rays, cull=False):
        """Closest instanced-mesh hit of rays [N, 8] (o, tmin, d, tmax): (out [N,4] t,u,v,hit; ids [N,2])."""
        r = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        out, ids = np.zeros((len(r), 4), np.float32), np.zeros((len(r), 2), np.int32)
        self._chk(self.lib.vxpt_mesh_probe(self.ctx, _ptr(r), len(r), int(bool(cull)), _ptr(out), _ptr(ids)),
                  "vxpt_mesh_probe")
        return out, ids

    def mesh_occluded(self, rays):
        """Visibility rays [N, 8] (o, tmin, d, tmax) against the instanced meshes, both faces:
        uint8 [N], 1 = some triangle lies in [tmin, tmax] (closesthit.cu:616-625)."""
        r = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        occ = np.zeros(len(r), np.uint8)
        self._chk(self.lib.vxpt_mesh_occluded(self.ctx, _ptr(r), len(r), _ptr(occ)), "vxpt_mesh_occluded")
        return occ

    def light_remap(self):
        """(previous -> current light index int32 [prevNumLights], pending: the next pass applies it)."""
        n, pend = ctypes.c_int(0), ctypes.c_int(0)
        self._chk(self.lib.vxpt_get_light_remap(self.ctx, None, 0, ctypes.byref(n), ctypes.byref(pend)),
                  "vxpt_get_light_remap")
        out = np.zeros(n.value, np.int32)
        if n.value:
            self._chk(self.lib.vxpt_get_light_remap(self.ctx, _ptr(out), n.value, None, None), "vxpt_get_light_remap")
        return out, bool(pend.value)

    def lights(self):
        """(mapping uint32 [M, 3], LightInfo records uint8 [L, 32], alias bins [L], local luminance)."""
        n, nl, lum = ctypes.c_int(0), ctypes.c_uint32(0), ctypes.c_float(0)
        self._chk(self.lib.vxpt_get_lights(self.ctx, None, 0, ctypes.byref(n), ctypes.byref(nl), ctypes.byref(lum)),
                  "vxpt_get_lights")
        mp = np.zeros((n.value, 3), np.uint32)
        if n.value:
            self._chk(self.lib.vxpt_get_lights(self.ctx, _ptr(mp), n.value, ctypes.byref(n), None, None),
                      "vxpt_get_lights")
        recs = np.zeros((nl.value, 32), np.uint8)
        bins = np.zeros(nl.value, ALIAS_DTYPE)
        if nl.value:
            self._chk(self.lib.vxpt_readback(self.ctx, BUF["LIGHTS"], _ptr(recs), recs.nbytes), "vxpt_readback")
            self._chk(self.lib.vxpt_readback(self.ctx, BUF["LIGHT_ALIAS"], _ptr(bins), bins.nbytes), "vxpt_readback")
        return mp, recs, bins, lum.value

    # --- voxel edits (VoxelEngine click path) and world files (WorldSceneManager) ---
    @staticmethod
    def _pick_dict(o):
        return dict(hit=bool(o[0]), hit_pos=tuple(int(v) for v in o[1:4]), hit_id=int(o[4]), space=bool(o[5]),
                    place_pos=tuple(int(v) for v in o[6:9]), cells=int(o[9]))

    def pick_block(self):
        o = np.zeros(10, np.int32)
        self._chk(self.lib.vxpt_pick_block(self.ctx, _ptr(o)), "vxpt_pick_block")
        return self._pick_dict(o)

    def set_block(self, x, y, z, block_id):
        self._chk(self.lib.vxpt_set_block(self.ctx, int(x), int(y), int(z), int(block_id)), "vxpt_set_block")

    def click_block(self, block_id):
        o = np.zeros(10, np.int32)
        self._chk(self.lib.vxpt_click_block(self.ctx, int(block_id), _ptr(o)), "vxpt_click_block")
        return self._pick_dict(o)

    def save_world(self, scene_yaml, chunk_dir):
        self._chk(self.lib.vxpt_save_world(self.ctx, str(scene_yaml).encode(), str(chunk_dir).encode()),
                  "vxpt_save_world")

    def load_world(self, scene_yaml, chunk_dir):
        cam = Camera()
        self._chk(self.lib.vxpt_load_world(self.ctx, str(scene_yaml).encode(), str(chunk_dir).encode(),
                                           ctypes.byref(cam)), "vxpt_load_world")
        if not hasattr(self, "chunks"):  # a fresh context takes the scene's chunk_config
            cfg = {}
            for line in open(scene_yaml):
                k, _, v = line.strip().partition(":")
                if k in ("chunksX", "chunksY", "chunksZ"):
                    cfg[k] = int(v)
            self.chunks = (cfg["chunksX"], cfg["chunksY"], cfg["chunksZ"])
        return cam

    # --- frame (OfflineBackend::renderFrame) ---
    def trace(self, iteration_index, primary_only=False):
        self._chk(self.lib.vxpt_trace(self.ctx, iteration_index, TRACE_PRIMARY_ONLY if primary_only else 0),
                  "vxpt_trace")

    def trace_flags(self, iteration_index, flags):
        """vxpt_trace with raw flags (VXPT_TRACE_ACCUMULATE | ACCUM_FIRST | spp << 8)."""
        self._chk(self.lib.vxpt_trace(self.ctx, iteration_index, flags), "vxpt_trace")

    # --- band partition (multi-GPU, bands.py) ---
    def set_band(self, y0, y1):
        self._chk(self.lib.vxpt_set_band(self.ctx, y0, y1), "vxpt_set_band")

    def row_bytes(self, name):
        n = self.lib.vxpt_row_bytes(self.ctx, BUF[name] if isinstance(name, str) else int(name))
        if n <= 0:
            raise VxptError("buffer %s has no row layout" % name)
        return n

    def copy_rows(self, name, y, rows, dev_ptr, to_buffer):
        which = BUF[name] if isinstance(name, str) else int(name)
        self._chk(self.lib.vxpt_copy_rows(self.ctx, which, y, rows, ctypes.c_void_p(dev_ptr), int(to_buffer)),
                  "vxpt_copy_rows")

    # --- post-processing + frame output (PostProcessor::run, OfflineBackend::writeFrameBufferToPNG) ---
    def denoise_params(self):
        """The settings file's denoiser parameters (what NULL params mean to the library)."""
        p = DenoiseParams()
        self._chk(self.lib.vxpt_get_denoise_params(self.ctx, ctypes.byref(p)), "vxpt_get_denoise_params")
        return p

    def post_params(self):
        p = PostParams()
        self._chk(self.lib.vxpt_get_post_params(self.ctx, ctypes.byref(p)), "vxpt_get_post_params")
        return p

    def postprocess(self, params=None, dt_ms=16.6667):
        self._chk(self.lib.vxpt_postprocess(self.ctx, ctypes.byref(params) if params is not None else None,
                                            float(dt_ms)), "vxpt_postprocess")

    def sun_projection(self):
        """(on_screen, px, py, u, v, accumulated sun luminance) of the lens flare."""
        o = np.zeros(6, np.float32)
        self._chk(self.lib.vxpt_get_sun_projection(self.ctx, o.ctypes.data), "vxpt_get_sun_projection")
        return bool(o[0]), int(o[1]), int(o[2]), float(o[3]), float(o[4]), float(o[5])

    def write_png(self, path):
        """The post-processed frame as the reference's offline PNG."""
        write_png(path, self.read("FRAME"))

    def band_gather(self, name, root=0):
        """vxpt_band_gather: every band's rows of `name` into the root rank's buffer (RCCL)."""
        self._chk(self.lib.vxpt_band_gather(self.ctx, BUF[name] if isinstance(name, str) else int(name), root),
                  "vxpt_band_gather")

    def exchange_halo(self, names, rows):
        """vxpt_exchange_halo: one RCCL halo exchange of the named buffers with the band neighbours."""
        mask = 0
        for n in names:
            mask |= 1 << (BUF[n] if isinstance(n, str) else int(n))
        self._chk(self.lib.vxpt_exchange_halo(self.ctx, mask, rows), "vxpt_exchange_halo")

    def band_comm_init(self, comm_id, nranks, rank, splits=None):
        """Attach an RCCL communicator (vxpt_band_comm_init): this context renders band `rank`
        of `nranks` and vxpt_render_frame exchanges the halos itself.  splits: the nranks + 1 row
        boundaries of an uneven partition (vxpt_band_comm_init_rows), the same on every rank."""
        buf = ctypes.create_string_buffer(bytes(comm_id), len(comm_id))
        if splits is None:
            self._chk(self.lib.vxpt_band_comm_init(self.ctx, buf, len(comm_id), nranks, rank), "vxpt_band_comm_init")
        else:
            s = _splits_array(splits, nranks)
            self._chk(self.lib.vxpt_band_comm_init_rows(self.ctx, buf, len(comm_id), nranks, rank, s.ctypes.data),
                      "vxpt_band_comm_init_rows")

    def denoise(self, frame_num, iteration_index, params=None):
        p = params or DenoiseParams.defaults()
        self._chk(self.lib.vxpt_denoise(self.ctx, ctypes.byref(p), frame_num, iteration_index), "vxpt_denoise")

    def denoise_pass(self, which, arg=0, arg2=0, params=None):
        p = params or DenoiseParams.defaults()
        self._chk(self.lib.vxpt_denoise_pass(self.ctx, ctypes.byref(p), which, arg, arg2), "vxpt_denoise_pass")

    def render_frame(self, frame_num, spp=1, params=None):
        p = params or DenoiseParams.defaults()
        self._chk(self.lib.vxpt_render_frame(self.ctx, ctypes.byref(p), frame_num, spp), "vxpt_render_frame")

    def render_frames(self, frame0, n_frames, spp=1, params=None):
        """vxpt_render_frames: frames frame0 .. frame0+n_frames-1 with the camera held, each frame's
        first trace pass overlapping the previous frame's last (same buffers as render_frame calls)."""
        p = params or DenoiseParams.defaults()
        self._chk(self.lib.vxpt_render_frames(self.ctx, ctypes.byref(p), frame0, n_frames, spp), "vxpt_render_frames")

    def tuning(self):
        t = Tuning()
        self._chk(self.lib.vxpt_get_tuning(self.ctx, ctypes.byref(t)), "vxpt_get_tuning")
        return t.as_dict()

    def set_tuning(self, **fields):
        """vxpt_set_tuning with the named fields changed (the rest as they are)."""
        t = Tuning()
        self._chk(self.lib.vxpt_get_tuning(self.ctx, ctypes.byref(t)), "vxpt_get_tuning")
        for k, v in fields.items():
            if k not in TUNING_FIELDS:
                raise VxptError("unknown tuning field " + k)
            setattr(t, k, int(v))
        self._chk(self.lib.vxpt_set_tuning(self.ctx, ctypes.byref(t)), "vxpt_set_tuning")

    def timings(self):
        t = Timing()
        self._chk(self.lib.vxpt_timings(self.ctx, ctypes.byref(t)), "vxpt_timings")
        return dict(trace_ms=t.trace_ms, denoise_ms=t.denoise_ms, sky_ms=t.sky_ms, frame_ms=t.frame_ms,
                    host_ms=t.host_ms)

    def debug_clamp_decisions(self, on=True):
        """vxpt_debug_clamp_decisions: the history clamp records its decision bits (CLAMP_DECISION)."""
        self._chk(self.lib.vxpt_debug_clamp_decisions(self.ctx, 1 if on else 0), "vxpt_debug_clamp_decisions")

    def band_stats_enable(self, on=True):
        """vxpt_band_stats_enable: halo-exchange / band-span collection on (totals reset) or off."""
        self._chk(self.lib.vxpt_band_stats_enable(self.ctx, 1 if on else 0), "vxpt_band_stats_enable")

    def band_stats(self):
        """vxpt_band_stats: the totals since the last enable, as a dict."""
        s = BandStat()
        self._chk(self.lib.vxpt_band_stats(self.ctx, ctypes.byref(s)), "vxpt_band_stats")
        return {f: getattr(s, f) for f, _ in s._fields_}

    def sync(self):
        self._chk(self.lib.vxpt_sync(self.ctx), "vxpt_sync")

    # --- buffers ---
    def _shape(self, which):
        n = self.W * self.H
        if which == BUF["RESERVOIRS"]:
            return np.zeros(2 * n, RESERVOIR_DTYPE)
        if which in (BUF["RES_EVEN"], BUF["RES_ODD"]):
            return np.zeros((self.H, self.W), RESERVOIR_DTYPE)
        if which == BUF["SKY"]:
            return np.zeros((512, 1024, 4), np.float32)
        if which == BUF["SUN"]:
            return np.zeros((32, 32, 4), np.float32)
        if which == BUF["VOXELS"]:
            cx, cy, cz = self.chunks
            return np.zeros(cx * cy * cz * 32768, np.uint8)
        if which == BUF["TEXELS"]:
            return np.zeros((self.texture_table()[1], 4), np.uint8)
        if which in (BUF["OCTANT_TABLES"], BUF["CELL_MASKS"], BUF["BRICK_IDS"], BUF["MACRO_MASKS"], BUF["BOX_TABLES"]):
            nb = int(np.prod(self.chunks)) * 512
            return {BUF["OCTANT_TABLES"]: np.zeros(8 * nb, np.uint8), BUF["CELL_MASKS"]: np.zeros(nb, np.uint64),
                    BUF["BOX_TABLES"]: np.zeros(8 * nb, np.uint32),
                    BUF["BRICK_IDS"]: np.zeros(nb * 64, np.uint8),
                    BUF["MACRO_MASKS"]: np.zeros(nb // 64, np.uint64)}[which]
        if which in FLOAT1_BUFS:
            return np.zeros((self.H, self.W), np.float32)
        if which == BUF["TAP_RECORD"]:
            return np.zeros((self.H, self.W, 8), np.float32)
        return np.zeros((self.H, self.W, 4), np.float32)

    def read(self, name):
        which = BUF[name] if isinstance(name, str) else int(name)
        out = self._shape(which)
        self._chk(self.lib.vxpt_readback(self.ctx, which, _ptr(out), out.nbytes), "vxpt_readback")
        return out

    def write(self, name, data):
        which = BUF[name] if isinstance(name, str) else int(name)
        ref = self._shape(which)
        data = np.ascontiguousarray(data, dtype=ref.dtype).reshape(ref.shape)
        self._chk(self.lib.vxpt_upload(self.ctx, which, _ptr(data), data.nbytes), "vxpt_upload")

    def sky_alias(self):
        n = 1024 * 512
        q, p = np.zeros(n, np.float32), np.zeros(n, np.float32)
        a, sd = np.zeros(n, np.int32), np.zeros(3, np.float32)
        self._chk(self.lib.vxpt_get_sky_alias(self.ctx, _ptr(q), _ptr(p), _ptr(a), _ptr(sd)), "vxpt_get_sky_alias")
        return q, p, a, sd

    def probe_rays(self, rays, mode=0):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        n = rays.shape[0]
        out = np.zeros((n, 6), np.int32)
        t = np.zeros(n, np.float32)
        self._chk(self.lib.vxpt_probe_rays(self.ctx, n, _ptr(rays), _ptr(out), _ptr(t), mode), "vxpt_probe_rays")
        return out, t

    def trace_counters(self):
        """Queue counters of the last trace pass: (16, 3) array of (rays queued,
        level-1 stragglers, level-2 stragglers) per queue 4*segment + kind."""
        out = np.zeros(48, np.uint32)
        self._chk(self.lib.vxpt_trace_counters(self.ctx, _ptr(out), 48), "vxpt_trace_counters")
        return out.reshape(16, 3)

    def upload_materials(self, mats):
        """mats: list of 12 dicts (block ids 1..12) with albedo, roughness, translucency,
        metallic, material_id, thinfilm (MaterialManager GPU table)."""
        arr = (Material * len(mats))()
        for i, m in enumerate(mats):
            arr[i] = Material((ctypes.c_float * 3)(*m.get("albedo", (1.0, 1.0, 1.0))), m.get("roughness", 0.8),
                              m.get("translucency", 0.0), int(m.get("metallic", 0)), m.get("material_id", i),
                              int(m.get("thinfilm", 0)))
        self._chk(self.lib.vxpt_upload_materials(self.ctx, arr, len(mats)), "vxpt_upload_materials")

    def probe_rng(self, queries):
        """queries: (n, 4) int32 of (px, py, iterationIndex, dim) -> n floats."""
        q = np.ascontiguousarray(queries, np.int32).reshape(-1, 4)
        out = np.zeros(len(q), np.float32)
        self._chk(self.lib.vxpt_probe_rng(self.ctx, len(q), _ptr(q), _ptr(out)), "vxpt_probe_rng")
        return out


def render_offline(width, height, frames, spp=1, chunks=(2, 1, 2), height_scale=32.0, device=0):
    """mainOffline.cpp flow: settings, terrain, camera from the scene yaml, sky, frame loop."""
    r = Renderer(width, height, device=device)
    r.load_settings()
    r.generate_terrain(chunks, height_scale=height_scale)
    r.load_models()  # VoxelEngine::init: the instanced meshes present under the data directory
    cam = r.scene_camera()
    r.set_camera(list(cam.pos), list(cam.dir), cam.fov_deg)
    r.set_sky()
    for f in range(frames):
        r.render_frame(f, spp)
    return r


def band_comm_id():
    """RCCL unique id for vxpt_band_comm_init (rank 0 makes it, the host broadcasts it)."""
    lib = load_library()
    buf = ctypes.create_string_buffer(128)
    if lib.vxpt_band_comm_id(buf, 128) != 0:
        raise VxptError("vxpt_band_comm_id failed")
    return buf.raw


def bvh_depth(boxes, leaf_max):
    """vxpt_bvh_depth: (deepest leaf, node count) of the mesh BVH builder over [N, 6] boxes
    (pure host function); None if it cannot keep the depth limit."""
    b = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
    d, n = ctypes.c_int(0), ctypes.c_int(0)
    r = load_library().vxpt_bvh_depth(b.ctypes.data, len(b), leaf_max, ctypes.byref(d), ctypes.byref(n))
    return None if r != 0 else (d.value, n.value)


def _splits_array(splits, nranks):
    s = np.ascontiguousarray(splits, np.int32)
    if s.shape != (nranks + 1,):
        raise VxptError("row splits: %d boundaries expected, got %s" % (nranks + 1, s.shape))
    return s


def equal_splits(height, nranks):
    """The equal bands' nranks + 1 row boundaries (vxpt_band_rows of every rank)."""
    return [0] + [band_rows(height, nranks, r)[1] for r in range(nranks)]


def band_balance(height, splits, band_ms, block_cost=None):
    """vxpt_band_balance: (new row boundaries, refined per-8-row-block cost) from the measured time
    of each band of the partition `splits` (pure host function, no GPU).  Pass the returned cost
    back in to refine the estimate over several measurements."""
    n = len(splits) - 1
    s = _splits_array(splits, n)
    ms = np.ascontiguousarray(band_ms, np.float32)
    if ms.shape != (n,):
        raise VxptError("band_ms: %d times expected" % n)
    cost = np.full((height + 7) // 8, -1.0, np.float32) if block_cost is None else \
        np.array(block_cost, np.float32).copy()
    out = np.zeros(n + 1, np.int32)
    if load_library().vxpt_band_balance(height, n, s.ctypes.data, ms.ctypes.data, cost.ctypes.data,
                                        out.ctypes.data) != 0:
        raise VxptError("vxpt_band_balance: bad arguments")
    return [int(v) for v in out], cost


def band_rows(height, nranks, rank):
    """vxpt_band_rows: (row_begin, row_end) of `rank` (pure host function, no GPU)."""
    y0, y1 = ctypes.c_int(0), ctypes.c_int(0)
    if load_library().vxpt_band_rows(height, nranks, rank, ctypes.byref(y0), ctypes.byref(y1)) != 0:
        raise VxptError("vxpt_band_rows: bad arguments")
    return y0.value, y1.value


def halo_plan(height, nranks, rank, rows):
    """vxpt_halo_plan as bands.halo_plan's dict: {peer: ((send y, n), (recv y, n))}."""
    out, n = np.zeros(10, np.int32), ctypes.c_int(0)
    if load_library().vxpt_halo_plan(height, nranks, rank, rows, out.ctypes.data, ctypes.byref(n)) != 0:
        raise VxptError("vxpt_halo_plan: bad arguments")
    e = out.reshape(2, 5)[:n.value]
    return {int(p): ((int(sy), int(sn)), (int(ry), int(rn))) for p, sy, sn, ry, rn in e}


def band_halo_rows(cur, prev, width, height, nranks, near=None):
    """vxpt_band_halo_rows: (trace rows, history rows) of a banded frame whose camera moved from
    prev to cur ((pos, dir, fov) each); None when the library refuses the motion.  With `near`
    (vxpt_band_halo_rows_near) the camera may also translate: every primary hit lies at least
    `near` from it."""
    def cam(c):
        return Camera((ctypes.c_float * 3)(*c[0]), (ctypes.c_float * 3)(*c[1]), c[2])
    t, h = ctypes.c_int(0), ctypes.c_int(0)
    if near is None:
        r = load_library().vxpt_band_halo_rows(ctypes.byref(cam(cur)), ctypes.byref(cam(prev)), width, height,
                                               nranks, ctypes.byref(t), ctypes.byref(h))
    else:
        r = load_library().vxpt_band_halo_rows_near(ctypes.byref(cam(cur)), ctypes.byref(cam(prev)), width, height,
                                                    nranks, float(near), ctypes.byref(t), ctypes.byref(h))
    if r == -4:  # VXPT_ERR_STATE
        return None
    if r != 0:
        raise VxptError("vxpt_band_halo_rows: bad arguments")
    return t.value, h.value


class LinkedBands:
    """n contexts of this process rendering the bands of one frame (vxpt_band_link):
    the library's multi-GPU schedule with device copies as the transport."""

    def __init__(self, renderers, splits=None):
        self.rs = list(renderers)
        self.lib = load_library()
        self._arr = (ctypes.c_void_p * len(self.rs))(*[r.ctx for r in self.rs])
        if splits is not None:
            s = _splits_array(splits, len(self.rs))
            rc = self.lib.vxpt_band_link_rows(self._arr, len(self.rs), s.ctypes.data)
        else:
            rc = self.lib.vxpt_band_link(self._arr, len(self.rs))
        if rc != 0:
            raise VxptError("vxpt_band_link: " + self.lib.vxpt_last_error(self.rs[0].ctx).decode())

    def render_frame(self, frame_num, spp=1, params=None):
        p = params or DenoiseParams.defaults()
        if self.lib.vxpt_render_frame_linked(self._arr, len(self.rs), ctypes.byref(p), frame_num, spp) != 0:
            raise VxptError("vxpt_render_frame_linked: " + self.lib.vxpt_last_error(self.rs[0].ctx).decode())

    def render_frames(self, frame0, n_frames, spp=1, params=None):
        """vxpt_render_frames_linked: the banded run's pipelined schedule over the linked bands."""
        p = params or DenoiseParams.defaults()
        if self.lib.vxpt_render_frames_linked(self._arr, len(self.rs), ctypes.byref(p), frame0, n_frames, spp) != 0:
            raise VxptError("vxpt_render_frames_linked: " + self.lib.vxpt_last_error(self.rs[0].ctx).decode())

    def gather(self, name, root=0):
        """vxpt_band_gather_linked: every band's rows of `name` into band `root`'s buffer."""
        if self.lib.vxpt_band_gather_linked(self._arr, len(self.rs), BUF[name] if isinstance(name, str) else int(name),
                                            root) != 0:
            raise VxptError("vxpt_band_gather_linked: " + self.lib.vxpt_last_error(self.rs[0].ctx).decode())

    def postprocess(self, params=None, dt_ms=16.6667):
        """vxpt_postprocess over the bands (histogram summed over them, 1-row and bloom halos)."""
        if self.lib.vxpt_postprocess_linked(self._arr, len(self.rs), ctypes.byref(params) if params is not None else None,
                                            float(dt_ms)) != 0:
            raise VxptError("vxpt_postprocess_linked: " + self.lib.vxpt_last_error(self.rs[0].ctx).decode())


def write_png(path, frame):
    """OfflineBackend::writeFrameBufferToPNG: H x W x 4 float32 -> 8-bit RGB PNG (clamped, x255, Y flip)."""
    lib = load_library()
    f = np.ascontiguousarray(frame, dtype=np.float32)
    if lib.vxpt_write_png_rgba32f(os.fsencode(path), f.shape[1], f.shape[0], f.ctypes.data) != 0:
        raise VxptError("vxpt_write_png_rgba32f(%s) failed" % path)


def read_png(path):
    lib = load_library()
    w, h, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    if lib.vxpt_read_png(os.fsencode(path), ctypes.byref(w), ctypes.byref(h), ctypes.byref(c), None, 0) != 0:
        raise VxptError("cannot read %s" % path)
    px = np.zeros((h.value, w.value, c.value), np.uint8)
    if lib.vxpt_read_png(os.fsencode(path), None, None, None, px.ctypes.data, px.size) != 0:
        raise VxptError("cannot read %s" % path)
    return px


def image_diff(a, b, diff_png=None):
    """ImageDiff::compare (+ generateDiffImage when diff_png is given)."""
    lib = load_library()
    r = ImageDiffResult()
    if lib.vxpt_image_diff(os.fsencode(a), os.fsencode(b), ctypes.byref(r)) != 0:
        raise VxptError("image diff failed: %s vs %s" % (a, b))
    if diff_png and lib.vxpt_image_diff_png(os.fsencode(a), os.fsencode(b), os.fsencode(diff_png)) != 0:
        raise VxptError("diff image failed")
    return {f: getattr(r, f) for f, _ in r._fields_}


def read_obj(path):
    """The library's OBJ reader (no GPU needed): (pos [T,3,3], uv [T,3,2])."""
    L = load_library()
    n = ctypes.c_int(0)
    if L.vxpt_read_obj(str(path).encode(), None, None, 0, ctypes.byref(n)) != 0:
        raise IOError("vxpt_read_obj failed: %s" % path)
    pos, uv = np.zeros((n.value, 3, 3), np.float32), np.zeros((n.value, 3, 2), np.float32)
    if n.value:
        L.vxpt_read_obj(str(path).encode(), _ptr(pos), _ptr(uv), n.value, ctypes.byref(n))
    return pos, uv
