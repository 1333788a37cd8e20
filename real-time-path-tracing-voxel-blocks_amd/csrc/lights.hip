// vxpt -- emissive-triangle light table for the instanced meshes.
//
// One thread per (instance, triangle) of an emissive block type's mesh:
//   world-space corners = the instance's 3x4 translation applied to the object-space
//   corners (applyTransform, VoxelEngine.cu:33-39, evaluated as written: the
//   rotation part is the identity, so the products are exact);
//   TriangleLight{base = v0, edge1 = v1 - v0, edge2 = v2 - v0}.Store() (Light.h:124-137);
//   weight = luminance(radiance) * area of TriangleLight::Create(record) (Light.h:85-122,
//   extractRadianceKernel VoxelEngine.cu:139-147): the alias table is built from the
//   decoded (quantised) light, as in the reference.
// Byte work (~100 B per light); the table is rebuilt when the instance set changes.
#include "vx_internal.hpp"

namespace vx {
namespace {

// __float2half_rn bits (the hardware conversion rounds to nearest even)
VX_D uint32_t f16_bits(float f) { return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)f); }
VX_D float f16_float(uint32_t b) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(b & 0xFFFFu)); }
VX_D float sgn_nz(float v) { return v >= 0.0f ? 1.0f : -1.0f; }

// ndirToOctUnorm32 (LinearMath.h:2117-2122 via ndirToOctSigned / octWrap, :2093-2113)
VX_D uint32_t oct_encode(V3 n) {
    const float inv = 1.0f / (fabsf(n.x) + fabsf(n.y) + fabsf(n.z));
    float px = n.x * inv, py = n.y * inv;
    if (n.z < 0.0f) {
        const float wx = (1.0f - fabsf(py)) * sgn_nz(px), wy = (1.0f - fabsf(px)) * sgn_nz(py);
        px = wx;
        py = wy;
    }
    px = saturate(px * 0.5f + 0.5f);
    py = saturate(py * 0.5f + 0.5f);
    return (uint32_t)(px * 65534.0f) | ((uint32_t)(py * 65534.0f) << 16);
}
// octToNdirUnorm32 / octToNdirSigned (LinearMath.h:2069-2089)
VX_D V3 oct_decode(uint32_t u) {
    float px = saturate((float)(u & 0xFFFFu) / 65534.0f), py = saturate((float)(u >> 16) / 65534.0f);
    px = px * 2.0f - 1.0f;
    py = py * 2.0f - 1.0f;
    V3 n(px, py, 1.0f - fabsf(px) - fabsf(py));
    const float t = fmaxf(0.0f, -n.z);
    n.x += n.x >= 0.0f ? -t : t;
    n.y += n.y >= 0.0f ? -t : t;
    return normalize(n);
}

__global__ __launch_bounds__(256) void k_tri_lights(const float *tri, int nTri, const int *inst, int nInst, V3 radiance,
                                                    LightInfo *out, float *weight) {
    const unsigned g = blockIdx.x * 256u + threadIdx.x;
    if (g >= (unsigned)nTri * (unsigned)nInst) return;
    const unsigned ii = g / (unsigned)nTri, ti = g % (unsigned)nTri;
    const float tx = (float)inst[ii * 3], ty = (float)inst[ii * 3 + 1], tz = (float)inst[ii * 3 + 2];
    V3 v[3];
    for (int k = 0; k < 3; ++k) {
        const float *p = tri + (size_t)ti * 9 + k * 3;
        v[k] = V3(1.0f * p[0] + 0.0f * p[1] + 0.0f * p[2] + tx, 0.0f * p[0] + 1.0f * p[1] + 0.0f * p[2] + ty,
                  0.0f * p[0] + 0.0f * p[1] + 1.0f * p[2] + tz);
    }
    const V3 e1 = v[1] - v[0], e2 = v[2] - v[0];
    // Store()
    LightInfo li;
    const V3 c = v[0] + (e1 + e2) / 3.0f;
    li.center[0] = c.x; li.center[1] = c.y; li.center[2] = c.z;
    li.scalars = f16_bits(length(e1)) | (f16_bits(length(e2)) << 16);
    li.radiance[0] = f16_bits(radiance.x) | (f16_bits(radiance.y) << 16);
    li.radiance[1] = f16_bits(radiance.z) | (f16_bits(0.0f) << 16);
    li.direction1 = oct_encode(normalize(e1));
    li.direction2 = oct_encode(normalize(e2));
    out[g] = li;
    // Create(li): decoded edges and radiance -> surface area -> weight
    const V3 d1 = oct_decode(li.direction1) * f16_float(li.scalars), d2 = oct_decode(li.direction2) * f16_float(li.scalars >> 16);
    const V3 rad(f16_float(li.radiance[0]), f16_float(li.radiance[0] >> 16), f16_float(li.radiance[1]));
    const float nl = length(cross(d1, d2));
    const float area = nl > 0.0f ? 0.5f * nl : 0.0f;
    weight[g] = luminance(rad) * area;
}

}  // namespace

hipError_t launch_tri_lights(const float *tri, int nTri, const int *inst, int nInst, V3 radiance, LightInfo *out,
                             float *weight, hipStream_t st) {
    const unsigned n = (unsigned)nTri * (unsigned)nInst;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_tri_lights, dim3((n + 255) / 256), dim3(256), 0, st, tri, nTri, inst, nInst, radiance, out,
                       weight);
    return hipGetLastError();
}

}  // namespace vx
