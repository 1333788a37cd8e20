// ORACLE (test infrastructure only): C entry points over the reference's own
// terrain noise generator, compiled from its sources where they lie
// (/root/reference/voxelengine/Noise.cpp + ext/PerlinNoise.hpp) into
// oracle/_ref/libref_noise.so.  Used only to pin the oracle's Perlin
// restatement (orc_scene.cpp Perlin) and to generate tests/golden/noise_ref.npz.
#include "Noise.h"

extern "C" {
// PerlinNoiseGenerator(octaves, seed).getNoise(x, y) for n points (VoxelSceneGen.cu:361)
void ref_noise(int octaves, unsigned seed, int n, const float *xy, float *out) {
    PerlinNoiseGenerator g(octaves, seed);
    for (int i = 0; i < n; ++i) out[i] = g.getNoise(xy[2 * i], xy[2 * i + 1]);
}
}
