// CPU test driver of the library's light-id remap (csrc/light_map.hpp, the code vxpt_host.cpp runs):
// reads a script from stdin and prints each update's remap table.
//   edit <instance id> <removed 0/1>
//   update <full 0/1> <prevN> <total> <m> (<id> <first> <count>) x m   -> prints "remap v0 v1 ..."
#include <iostream>
#include <string>

#include "light_map.hpp"

int main() {
    vx::LightUpdateState st;
    std::string cmd;
    while (std::cin >> cmd) {
        if (cmd == "edit") {
            uint32_t id;
            int removed;
            std::cin >> id >> removed;
            st.incremental = true;
            (removed ? st.removed : st.changed).insert(id);
        } else if (cmd == "update") {
            int full;
            unsigned prevN, total, m;
            std::cin >> full >> prevN >> total >> m;
            std::vector<uint32_t> map(3 * m);
            for (auto &v : map) std::cin >> v;
            if (full) st.incremental = false;
            const std::vector<int> r = vx::light_id_map(st, map, prevN, total);
            std::cout << "remap";
            for (int v : r) std::cout << ' ' << v;
            std::cout << '\n';
        }
    }
    return 0;
}
