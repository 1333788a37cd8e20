// CPU test driver (host code only, no kernel launch): the library's temporal accumulation
// (denoise.hip temporal_px, with the packed world-position plane of wpos_px) or history clamping
// (history_clamp_px with its moments read from the planes) on planes dumped from the oracle.
// Usage: denoise_driver state.bin out.bin
//   state.bin: int32 W, H, mode (0 temporal, 1 clamping); 32 f32 camera, 32 f32 previous camera
//   (oracle camera_info layout); 9 f32 + 6 int32 denoiser parameters; then the planes, W*H each:
//   float4 illum, normalRough, motion, prevNormalRough, prevIllum, prevFast, ping, pong;
//   float depth, material, prevDepth, histLen, prevHistLen
//   out.bin: mode 0: float4 ping, float4 pong, float histLen; mode 1: float4 prevIllum, prevFast,
//   float prevHistLen
#include <cstdio>
#include <cstring>
#include <vector>

#include "denoise.hip"

using namespace vx;

static CamDev cam_from(const float *v) {
    CamDev c{};
    c.pos = V3(v[0], v[1], v[2]);
    c.dir = V3(v[3], v[4], v[5]);
    std::memcpy(&c.uvToWorld, v + 6, 36);
    std::memcpy(&c.worldToUv, v + 15, 36);
    c.res = V2(v[24], v[25]);
    c.invRes = V2(v[26], v[27]);
    c.tanHalfFov = V2(v[28], v[29]);
    return c;
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    int32_t hdr[3];
    float cams[64], fl[9];
    int32_t in[6];
    if (fread(hdr, 4, 3, f) != 3 || fread(cams, 4, 64, f) != 64 || fread(fl, 4, 9, f) != 9 || fread(in, 4, 6, f) != 6)
        return 1;
    const int W = hdr[0], H = hdr[1], mode = hdr[2];
    const size_t n = (size_t)W * H;
    std::vector<float4> illum(n), normalRough(n), motion(n), prevNormalRough(n), prevIllum(n), prevFast(n), ping(n),
        pong(n), wpos(n);
    std::vector<float> depth(n), material(n), prevDepth(n), histLen(n), prevHistLen(n);
    for (auto *v : {&illum, &normalRough, &motion, &prevNormalRough, &prevIllum, &prevFast, &ping, &pong})
        if (fread(v->data(), 16, n, f) != n) return 1;
    for (auto *v : {&depth, &material, &prevDepth, &histLen, &prevHistLen})
        if (fread(v->data(), 4, n, f) != n) return 1;
    fclose(f);
    DenoiseArgs a{};
    a.W = W; a.H = H; a.y0 = 0; a.y1 = H;
    a.cam = cam_from(cams);
    a.prevCam = cam_from(cams + 32);
    a.p = {fl[0], fl[1], fl[2], fl[3], fl[4], fl[5], fl[6], fl[7], fl[8], in[0], in[1], in[2], in[3], in[4], in[5]};
    a.illum = illum.data(); a.normalRough = normalRough.data(); a.motion = motion.data();
    a.depth = depth.data(); a.material = material.data();
    a.prevNormalRough = prevNormalRough.data(); a.prevDepth = prevDepth.data();
    a.ping = ping.data(); a.pong = pong.data(); a.prevIllum = prevIllum.data(); a.prevFast = prevFast.data();
    a.histLen = histLen.data(); a.prevHistLen = prevHistLen.data();
    a.wpos = wpos.data();
    // fill_denoise's launch-uniform terms (vxpt_host.cpp)
    a.invW = 1.0f / (float)W; a.invH = 1.0f / (float)H;
    a.thrB = a.p.disocclusionThreshold + (1.5f / (float)H);
    a.thrA = a.p.disocclusionThresholdAlternate + (1.5f / (float)H);
    a.frustumK = a.cam.tanHalfFov.x / (a.cam.res.x / 2);
    a.invAcc1 = 1.0f / (a.p.maxAcc + 1.0f);
    a.invFast1 = 1.0f / (a.p.maxFast + 1.0f);
    FILE *fo = fopen(argv[2], "wb");
    if (!fo) return 1;
    if (mode == 0) {
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) wpos[(size_t)y * W + x] = wpos_px(a, x, y, depth[(size_t)y * W + x]);
        const Qt rot = q_rotation_between(a.prevCam.dir, a.cam.dir);
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) temporal_px(a, rot, x, y, nullptr);
        fwrite(ping.data(), 16, n, fo);
        fwrite(pong.data(), 16, n, fo);
        fwrite(histLen.data(), 4, n, fo);
    } else {
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) history_clamp_host(a, x, y);
        fwrite(prevIllum.data(), 16, n, fo);
        fwrite(prevFast.data(), 16, n, fo);
        fwrite(prevHistLen.data(), 4, n, fo);
    }
    fclose(fo);
    return 0;
}
