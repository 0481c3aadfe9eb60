// Host check of the packed-inverse layout (csrc/layout.h): slot_of inverts
// slot_ij and the 4656 slots cover the upper triangle of 96x96 exactly once.
#define __host__
#define __device__
#include <cstdio>
#include <vector>

#include "layout.h"

int main() {
    std::vector<int> seen(96 * 96, 0);
    for (int o = 0; o < 4656; ++o) {
        int i, j;
        mas::slot_ij(o, i, j);
        if (i > j || i < 0 || j >= 96) { std::printf("bad ij %d\n", o); return 1; }
        if (seen[i * 96 + j]++) { std::printf("dup %d %d\n", i, j); return 1; }
        if (mas::slot_of(i, j) != o || mas::slot_of(j, i) != o) {
            std::printf("slot_of(%d,%d)=%d != %d\n", i, j, mas::slot_of(i, j), o);
            return 1;
        }
    }
    for (int i = 0; i < 96; ++i)
        for (int j = i; j < 96; ++j)
            if (seen[i * 96 + j] != 1) { std::printf("missing %d %d\n", i, j); return 1; }
    return 0;
}
