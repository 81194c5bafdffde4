// Diagnostic: what a hipIpcMemHandle_t holds across allocate / export /
// free cycles (do handle bytes repeat for different allocations?).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

static void dump(const char *what, const hipIpcMemHandle_t &h) {
    const unsigned char *b = reinterpret_cast<const unsigned char *>(&h);
    printf("%-28s", what);
    for (size_t i = 0; i < sizeof(h); ++i) printf("%02x%s", b[i], (i % 8 == 7) ? " " : "");
    printf("\n");
}

int main() {
    hipIpcMemHandle_t h[8];
    void *p[8] = {};
    const size_t sz[8] = {32u << 20, 64u << 20, 32u << 20, 32u << 20,
                          64u << 20, 128u << 20, 32u << 20, 32u << 20};
    // 0: alloc+export, 1: alloc+export, free 0, 2: alloc (32) ...
    for (int i = 0; i < 8; ++i) {
        if (hipMalloc(&p[i], sz[i]) != hipSuccess) return 1;
        if (hipIpcGetMemHandle(&h[i], p[i]) != hipSuccess) return 2;
        char name[64];
        snprintf(name, sizeof(name), "alloc %d (%zu MiB) %p", i, sz[i] >> 20, p[i]);
        dump(name, h[i]);
        if (i >= 1) { hipFree(p[i - 1]); p[i - 1] = nullptr; }
    }
    hipIpcMemHandle_t again;
    hipIpcGetMemHandle(&again, p[7]);
    dump("alloc 7 re-export", again);
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < i; ++j)
            if (memcmp(&h[i], &h[j], sizeof(h[i])) == 0) printf("IDENTICAL handles %d and %d\n", j, i);
    printf("done\n");
    return 0;
}
