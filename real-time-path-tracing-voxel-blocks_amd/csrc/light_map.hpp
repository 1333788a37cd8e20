// vxpt -- the light-id remap of a light update (host only, no HIP): VoxelEngine::updateLight's
// buildLightIdMapping (VoxelEngine.cu:503-539) and buildIncrementalLightMapping (:541-633).
// Shared by vxpt_host.cpp and the CPU test driver (tests/native/light_map_driver.cpp).
#pragma once
#include <cstdint>
#include <map>
#include <set>
#include <utility>
#include <vector>

namespace vx {

// Scene's light-update state (Scene.h:91-115)
struct LightUpdateState {
    bool incremental = false;                 // m_lightUpdateType == INCREMENTAL (sticky until a full update)
    std::set<uint32_t> changed, removed;      // m_changedInstances / m_removedInstances
    std::map<uint32_t, std::pair<uint32_t, uint32_t>> range;  // m_instanceToLightRange
};

// The previous -> current light index table of an update from prevN lights to a table whose
// emissive instances are `lightMap` (instance id, first light, count) triples, total lights in all:
// every previous light unmapped (-1); for an incremental update a light keeps its position within
// its instance's run unless the instance was removed or changed -- the instance -> range table is
// only refreshed by an incremental update, so the first one after a full build maps nothing.  The
// edit sets are cleared only when there were previous lights.
inline std::vector<int> light_id_map(LightUpdateState &st, const std::vector<uint32_t> &lightMap, unsigned prevN,
                                     unsigned total) {
    std::vector<int> remap(prevN, -1);
    if (prevN == 0) return remap;
    if (st.incremental) {
        std::map<uint32_t, std::pair<uint32_t, uint32_t>> cur;
        for (size_t k = 0; k + 2 < lightMap.size(); k += 3) cur[lightMap[k]] = {lightMap[k + 1], lightMap[k + 2]};
        std::vector<int64_t> owner(prevN, -1);
        for (const auto &e : st.range)
            for (uint32_t i = 0; i < e.second.second; ++i)
                if ((uint64_t)e.second.first + i < prevN) owner[e.second.first + i] = e.first;
        for (unsigned p = 0; p < prevN; ++p) {
            if (owner[p] < 0) continue;
            const uint32_t id = (uint32_t)owner[p];
            if (st.removed.count(id) || st.changed.count(id)) continue;
            const auto it = cur.find(id);
            if (it == cur.end()) continue;
            const auto &pr = st.range[id];
            const uint32_t rel = p - pr.first;
            if (rel < pr.second && rel < it->second.second && (uint64_t)it->second.first + rel < total)
                remap[p] = (int)(it->second.first + rel);
        }
        st.range = cur;
    }
    st.changed.clear();
    st.removed.clear();
    return remap;
}

}  // namespace vx
