// ORACLE (test infrastructure only): scene-side restatements --
// terrain generator, camera, blue-noise sampler, voxel traversal.
#pragma once
#include <cstdint>
#include <vector>
#include "orc_math.h"

namespace orc {

// ---------------------------------------------------------------- terrain
// siv::BasicPerlinNoise<float> (voxelengine/ext/PerlinNoise.hpp, MIT,
// v3.0.0 as vendored) restated: mt19937-driven Fisher-Yates-style shuffle of
// 0..255 (:229-244, :409-414), 3-D gradient noise with z fixed to 0.34567
// (:441-494), octave2D_01 (:314-330, :565-568).
struct Perlin {
    uint8_t perm[256];
    explicit Perlin(uint32_t seed);
    float noise3(float x, float y, float z) const;
    float octave2d_01(float x, float y, int octaves, float persistence = 0.5f) const;
};

// Voxel world: chunk-major u8 ids, 32^3 per chunk, linear id x + 32*(z + 32*y)
// (VoxelMath.h:120-127), chunk index cx + cX*(cz + cZ*cy) (VoxelSceneGen.cu:353-355).
struct World {
    int cx = 0, cy = 0, cz = 0;     // chunk counts
    std::vector<uint8_t> ids;       // cx*cy*cz*32768
    int wx() const { return cx * 32; }
    int wy() const { return cy * 32; }
    int wz() const { return cz * 32; }
    uint8_t at(int x, int y, int z) const {
        int c = (x >> 5) + cx * ((z >> 5) + cz * (y >> 5));
        return ids[(size_t)c * 32768 + (x & 31) + 32 * ((z & 31) + 32 * (y & 31))];
    }
};

// initVoxelsMultiChunk + GenerateVoxelChunk (VoxelSceneGen.cu:61-165, 341-388).
// heightScale = chunk width (32) in the reference; freqDen = global width.
// useFma: emulate nvcc --fmad=true contraction of `noise*1.4f - 0.7f`.
void generate_terrain(World &w, int cx, int cy, int cz, float heightScale, float freqDen, bool useFma,
                      bool keepShaderBalls, bool globalY = false);

// ---------------------------------------------------------------- camera
// Camera (shaders/Camera.h:6-150) as set up by mainOffline.cpp:227-251.
struct Camera {
    F2 res, invRes, tanHalfFov;
    F3 pos, dir;
    float yaw = 0, pitch = 0;
    M3 uvToWorld, worldToUv;
    void init(int w, int h);
    void update_matrices();
    F3 uv_to_dir(const F2 &uv) const { return normalize(uvToWorld * F3(uv.x, uv.y, 1.0f)); }
    F2 dir_to_uv(const F3 &d) const {
        F3 n = worldToUv * d;
        return F2(n.x / n.z, n.y / n.z);
    }
    float pixel_world_size_scale() const { return tanHalfFov.x / (res.x / 2); }
};
F3 yaw_pitch_to_dir(float yaw, float pitch);
// Full offline set-up: pos/dir/fov from the scene YAML -> yaw/pitch -> matrices
Camera make_offline_camera(int w, int h, F3 pos, F3 dir, float fovDeg);

// ---------------------------------------------------------------- sampler
// BlueNoiseRandGenerator::rand (RandGen.h:21-45), SPP=4 tables.
// The reference indexes rankingTile with `dim` (not dim%8, :30); the index can
// run past the 128 KiB table at pixel (127,127) -- defined here as wrapping
// modulo the table size.
struct BlueNoise {
    std::vector<uint8_t> sobol, scramble, rank;
    bool load(const char *dir);
    float rand(int i, int j, int s, int d) const {
        i &= 127; j &= 127; s &= 255;
        int rk = s ^ rank[(d + (i + j * 128) * 8) & (128 * 128 * 8 - 1)];
        int v = sobol[d + rk * 256];
        v ^= scramble[(d % 8) + (i + j * 128) * 8];
        return v / 256.0f;
    }
};

// ---------------------------------------------------------------- traversal
// Hit record of the voxel DDA.  face: 0 Up,1 Down,2 Left,3 Right,4 Back,5 Front
// (VoxelSceneGen.cu:13-58).
struct Hit {
    bool hit = false;
    int x = 0, y = 0, z = 0, face = -1, id = 0;
    float t = kRayMax;
};
inline bool is_cube(uint8_t id) { return id >= 1 && id <= 12; }
// Radiance rays: closest front face (CULL_BACK, RayGen.cu:52).  Visibility rays:
// any face in [tmin, tmax] (closesthit.cu:616-625, no culling).
Hit dda_closest(const World &w, const F3 &o, const F3 &d, float tmax);
bool dda_occluded(const World &w, const F3 &o, const F3 &d, float tmin, float tmax);
// Brute-force triangle caster over the face mesh the reference builds
// (MarkValidFaces/CompactMesh, VoxelSceneGen.cu:167-287) -- the independent
// definition of what OptiX + CULL_BACK returns; used to pin dda_closest.
Hit mesh_closest(const World &w, const F3 &o, const F3 &d, float tmax);

// Self-intersection-safe spawn points for a cube-face hit (SelfHit.h:539-656
// specialised to axis-aligned unit quads under one translation instance).
void safe_spawn(const Hit &h, const F3 &hitPos, F3 &front, F3 &back, F3 &geoNormal);
F3 face_normal(int face);

}  // namespace orc
