// What is inside a hipIpcMemHandle_t on this runtime (dmabuf IPC mode)?
// Prints the raw handle words of a few allocations, a second export of the
// same allocation, and an export after a free, next to this process's pid
// and its open dmabuf file descriptors — to see whether the handle carries
// an exporter fd number (which the kernel reuses after a close).
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

static void dump(const char *what, const void *p) {
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, const_cast<void *>(p));
    unsigned w[16];
    memcpy(w, &h, sizeof(w));
    printf("%-22s %p rc=%d :", what, p, (int)e);
    for (int i = 0; i < 16; ++i) printf(" %08x", w[i]);
    printf("\n");
}

static void fds(const char *when) {
    printf("fds %s:", when);
    DIR *d = opendir("/proc/self/fd");
    if (!d) return;
    while (dirent *x = readdir(d)) {
        if (x->d_name[0] == '.') continue;
        char path[64], tgt[256] = {0};
        snprintf(path, sizeof(path), "/proc/self/fd/%s", x->d_name);
        if (readlink(path, tgt, sizeof(tgt) - 1) > 0 && strstr(tgt, "dmabuf")) printf(" %s", x->d_name);
    }
    closedir(d);
    printf("\n");
}

int main() {
    printf("pid %d (0x%x)\n", (int)getpid(), (unsigned)getpid());
    const size_t sz = 4u << 20;
    void *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
    (void)hipMalloc(&a, sz);
    (void)hipMalloc(&b, sz);
    (void)hipMalloc(&c, sz);
    fds("after alloc");
    dump("A", a);
    dump("A again", a);
    dump("B", b);
    dump("C", c);
    dump("A+1MiB", (char *)a + (1 << 20));
    fds("after exports");
    (void)hipFree(b);
    fds("after free B");
    (void)hipMalloc(&d, sz);
    dump("D (after free B)", d);
    dump("C again", c);
    fds("end");
    (void)hipFree(a);
    (void)hipFree(c);
    (void)hipFree(d);
    return 0;
}
