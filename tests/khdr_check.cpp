// Round trip of the k_gemm / k_dwl launch header packing (sacx_internal.h: khdr_of / khdr_field)
// against random launch geometries; built and run by tests/test_abi.py::test_launch_header_round_trip
#include "sacx_internal.h"
#include <cstdio>
#include <random>
using namespace sacx;
int main() {
    std::mt19937 r(1);
    int bad = 0;
    for (int it = 0; it < 200000; ++it) {
        GemmArgs a{};
        a.nprob = 1 + r() % 8; a.has_final = r() % 3; a.xcd_map = r() % 2;
        a.total_tiles = r() % 4096; a.row_blocks = r() % 1024;
        for (int i = 0; i < 8; ++i) a.probs[i].tile_begin = r() % 4096;
        if (it % 7 == 0) a.total_tiles = 5000;   // invalid
        KHdr k = khdr_of(a);
        const uint32_t f = khdr_flags(k);
        const bool valid = (f & 0x80u) != 0;
        if (a.total_tiles > 4095) { bad += valid; continue; }
        if (!valid) { bad++; continue; }
        bad += (int)khdr_field(k, 0) != a.total_tiles;
        bad += (int)khdr_field(k, 1) != a.row_blocks;
        for (int i = 1; i < a.nprob; ++i) bad += (int)khdr_field(k, i + 1) != a.probs[i].tile_begin;
        bad += (int)(f & 15) != a.nprob; bad += (int)((f >> 4) & 3) != a.has_final; bad += (int)((f >> 6) & 1) != a.xcd_map;
    }
    printf("khdr round trip: %d mismatches\n", bad);
    return bad != 0;
}
