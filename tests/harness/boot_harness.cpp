// CPU-only multi-process check of the shared-memory rendezvous
// (ompi_amd/csrc/bootstrap.cpp), linked against libompi_amd.so.
// usage: boot_harness <name> <rank> <size> <iters>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../ompi_amd/csrc/bootstrap.h"

int main(int argc, char **argv) {
    if (argc < 5) return 2;
    const int rank = atoi(argv[2]), size = atoi(argv[3]), iters = atoi(argv[4]);
    ompi_amd::ShmBoot boot;
    if (boot.attach(argv[1], rank, size, 30.0) != 0) { fprintf(stderr, "attach failed\n"); return 3; }
    for (int it = 0; it < iters; ++it) {
        // variable-length blobs, every byte checked
        const size_t len = 1 + (size_t)((it * 37) % ompi_amd::ShmBoot::kBlob);
        static unsigned char mine[ompi_amd::ShmBoot::kBlob], all[16 * ompi_amd::ShmBoot::kBlob];
        for (size_t i = 0; i < len; ++i) mine[i] = (unsigned char)(rank * 31 + it * 7 + i);
        if (boot.allgather(mine, all, len) != 0) { fprintf(stderr, "allgather failed\n"); return 4; }
        for (int r = 0; r < size; ++r)
            for (size_t i = 0; i < len; ++i)
                if (all[r * len + i] != (unsigned char)(r * 31 + it * 7 + i)) {
                    fprintf(stderr, "mismatch rank %d iter %d byte %zu\n", r, it, i);
                    return 5;
                }
        if ((it % 5) == 0 && boot.barrier() != 0) return 6;
    }
    printf("ok %d\n", rank);
    return 0;
}
