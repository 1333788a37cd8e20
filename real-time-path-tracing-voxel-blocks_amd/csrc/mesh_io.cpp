// vxpt -- Wavefront OBJ reader for the instanced block meshes.
//
// Behaviour of the reference's ObjUtils::extractMeshFromOBJ (renderer/assets/
// ObjUtils.cpp:13-120), which ModelManager::loadOBJModel (ModelManager.cpp:172-226)
// turns into one vertex per face corner:
//   - `v x y z` and `vt u v` lines are collected; everything else is ignored
//     (normals included: the renderer derives the geometric normal);
//   - `f` takes its first three corners only (the meshes are triangulated);
//     a corner is `v`, `v/t`, `v//n` or `v/t/n`; indices are 1-based, an index
//     below 1 (also negative / relative ones) clamps to the first element, a
//     missing texture index reads as element 0;
//   - a corner that does not start with an integer fails the whole file;
//   - the output is expanded: corner k of triangle j is vertex 3j+k, its position
//     and texcoord copied from the tables (out-of-range index -> zeros).
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/vxpt.h"
#include "vx_internal.hpp"

namespace vx {
namespace {

// whitespace-separated tokens of one line
std::vector<std::string> tokens(const std::string &line) {
    std::vector<std::string> t;
    size_t i = 0;
    while (i < line.size()) {
        while (i < line.size() && std::isspace((unsigned char)line[i])) ++i;
        size_t j = i;
        while (j < line.size() && !std::isspace((unsigned char)line[j])) ++j;
        if (j > i) t.emplace_back(line.substr(i, j - i));
        i = j;
    }
    return t;
}

// a stream-extracted float: the longest valid prefix, 0 when there is none
float to_float(const std::string &s) {
    const char *b = s.c_str();
    char *e = nullptr;
    const float v = std::strtof(b, &e);
    return e == b ? 0.0f : v;
}

// leading integer of s starting at pos; false when there is none
bool read_int(const std::string &s, size_t &pos, long &out) {
    const char *b = s.c_str() + pos;
    char *e = nullptr;
    const long v = std::strtol(b, &e, 10);
    if (e == b) return false;
    out = v;
    pos += (size_t)(e - b);
    return true;
}

}  // namespace

bool load_obj(const std::string &path, std::vector<float> &pos, std::vector<float> &uv) {
    std::ifstream f(path);
    if (!f) return false;
    std::vector<float> vp, vt;
    std::vector<unsigned> pi, ti;
    std::string line;
    while (std::getline(f, line)) {
        const std::vector<std::string> t = tokens(line);
        if (t.empty()) continue;
        if (t[0] == "v") {
            for (int k = 0; k < 3; ++k) vp.push_back(k + 1 < (int)t.size() ? to_float(t[k + 1]) : 0.0f);
        } else if (t[0] == "vt") {
            for (int k = 0; k < 2; ++k) vt.push_back(k + 1 < (int)t.size() ? to_float(t[k + 1]) : 0.0f);
        } else if (t[0] == "f") {
            for (int k = 0; k < 3 && k + 1 < (int)t.size(); ++k) {
                const std::string &c = t[k + 1];
                size_t p = 0;
                long v = 0, tx = 0;
                if (!read_int(c, p, v)) return false;
                if (p < c.size() && c[p] == '/') ++p;
                if (p >= c.size() || c[p] != '/') {
                    if (!read_int(c, p, tx)) tx = 0;
                }
                v -= 1;
                tx -= 1;
                pi.push_back((unsigned)(v < 0 ? 0 : v));
                ti.push_back((unsigned)(tx < 0 ? 0 : tx));
            }
        }
    }
    const size_t n = pi.size(), np = vp.size() / 3, nt = vt.size() / 2;
    pos.assign(n * 3, 0.0f);
    uv.assign(n * 2, 0.0f);
    for (size_t i = 0; i < n; ++i) {
        if (pi[i] < np)
            for (int k = 0; k < 3; ++k) pos[i * 3 + k] = vp[(size_t)pi[i] * 3 + k];
        if (ti[i] < nt)
            for (int k = 0; k < 2; ++k) uv[i * 2 + k] = vt[(size_t)ti[i] * 2 + k];
    }
    return true;
}

}  // namespace vx

extern "C" int vxpt_read_obj(const char *path, float *pos, float *uv, int cap_triangles, int *n_triangles) {
    if (!path) return VXPT_ERR_ARG;
    std::vector<float> p, t;
    if (!vx::load_obj(path, p, t)) return VXPT_ERR_IO;
    const int n = (int)(p.size() / 9);
    if (n_triangles) *n_triangles = n;
    const int m = n < cap_triangles ? n : cap_triangles;
    for (int i = 0; pos && i < m * 9; ++i) pos[i] = p[i];
    for (int i = 0; uv && i < m * 6; ++i) uv[i] = t[i];
    return VXPT_OK;
}
