// ORACLE (test infrastructure only): spectral sky/sun model + alias tables.
#pragma once
#include <vector>
#include "orc_math.h"

namespace orc {

struct AliasBin { float q, p; int alias; };

// Vose alias table, CPU build path (AliasTable.cu:66-153) with the weight sum
// defined as a sequential binary32 sum over i = 0..n-1 (the reference uses an
// order-unspecified thrust::reduce).
std::vector<AliasBin> build_alias(const std::vector<float> &weights, float &sum);
// AliasTable::sample (AliasTable.h:34-51)
inline unsigned alias_sample(const std::vector<AliasBin> &b, float u, float &pmf) {
    const int len = (int)b.size();
    int offset = mymin(int(u * len), int(len - 1));
    float up = mymin(u * len - offset, 0.999999f);
    if (up < b[offset].q) { pmf = b[offset].p; return offset; }
    int a = b[offset].alias;
    pmf = b[a].p;
    return a;
}

struct Sky {
    int skyW = 1024, skyH = 512, sunW = 32, sunH = 32;   // Sky.h:53-54
    F3 sunDir;
    std::vector<float> sky;   // skyW*skyH*4 (float4 texels, w = 0)
    std::vector<float> sun;   // sunW*sunH*4
    std::vector<AliasBin> skyAlias, sunAlias;
    float skySum = 0, sunSum = 0;
    bool load_tables(const char *dir);
    // SkyModel::update (Sky.cu:355-396)
    void build(float timeOfDay, float sunAxisAngleDeg, float sunAxisRotateDeg, float brightness);
    std::vector<float> tSky, tSkyRad, tSolar, tLimb;
};

}  // namespace orc
