// Host check of the t16 slot and slab maps of nrc_internal.h (no GPU): run by tests/test_layouts.py.
// Frequency and Hash (round 5): every canonical feature in exactly one layer-0 K slot, every MLP parameter at exactly one
// slab position (closed forms t16_slab_param / t16_hash_slab_param), the Hash W0^T fragments 36..39 without collisions.
#include <cstdio>
#include <vector>

#include "nrc_internal.h"

using namespace nrc_amd;

static int fail(const char* what, int a, int b) {
    std::printf("FAIL %s (%d, %d)\n", what, a, b);
    return 1;
}

int main() {
    for (int hash = 0; hash < 2; ++hash) {
        const int in0 = hash ? NRC_HASH_ENC_WIDTH : NRC_ENC_WIDTH, nparam = hash ? NRC_HASH_MLP_PARAMS : NRC_NUM_PARAMS;
        std::vector<int> seen(in0, 0);
        for (int K = 0; K < 96; ++K) {
            const int f = hash ? t16_hash_slot_feature(K) : t16_slot_feature(K);
            if (f < -1 || f >= in0) return fail("slot feature range", K, f);
            if (f >= 0) ++seen[f];
        }
        for (int f = 0; f < in0; ++f)
            if (seen[f] != 1) return fail("feature not in exactly one slot", f, seen[f]);
        std::vector<int> hit(nparam, 0);
        for (int pos = 0; pos < slab_floats(0); ++pos) {
            const int p = hash ? t16_hash_slab_param(pos) : t16_slab_param(pos);
            if (p < -1 || p >= nparam) return fail("slab param range", pos, p);
            if (p >= 0) ++hit[p];
        }
        for (int p = 0; p < nparam; ++p)
            if (hit[p] != 1) return fail("parameter not at exactly one slab position", p, hit[p]);
    }
    // Hash W0^T of the grid features: (frag 36 + 2 mb + s, lane 16 g + m, element j) unique over (row o, grid slot f)
    std::vector<int> used(4 * 64 * 8, 0);
    for (int o = 0; o < 64; ++o)
        for (int f = 0; f < 2 * NRC_HASH_LEVELS; ++f) {
            const int s = o >> 5, g = (o >> 2) & 3, j = 4 * ((o >> 4) & 1) + (o & 3);
            if (t16_row(s, g, j) != o) return fail("t16_row inverse", o, t16_row(s, g, j));
            const int idx = ((2 * (f >> 4) + s) * 64 + 16 * g + (f & 15)) * 8 + j;
            if (used[idx]++) return fail("W0^T fragment collision", o, f);
        }
    std::printf("t16 maps OK\n");
    return 0;
}
