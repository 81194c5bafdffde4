// Two exporters, one importer: can a handle of exporter E2 be answered with
// a mapping of exporter E1's buffer when both buffers sit at the same
// virtual address in their own processes (ranks that allocate in the same
// order on one device get the same addresses)?
//   E1, E2 (children, forked before any HIP call) each allocate a buffer of
//   the same size, fill it with their own byte and send the handle.
//   The importer opens E1's handle, then E2's, and reads one byte of each.
// Per round the exporters free and re-allocate (same address again) and the
// importer closes (scenario "close") or keeps (scenario "keep", closed one
// round later) its previous mappings.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

static const size_t kSize = 8u << 20;

struct reply {
    hipIpcMemHandle_t h;
    void *va;
};

static void wr(int fd, const void *p, size_t n) {
    if (write(fd, p, n) != (ssize_t)n) _exit(3);
}
static void rd(int fd, void *p, size_t n) {
    size_t got = 0;
    while (got < n) {
        ssize_t k = read(fd, (char *)p + got, n - got);
        if (k <= 0) _exit(4);
        got += (size_t)k;
    }
}

// exporter: on each request byte, free the old buffer, allocate a new one,
// fill it with `fill`, reply with its handle and address; 0 = quit
static void exporter(int in, int out, unsigned char fill) {
    void *buf = nullptr;
    for (;;) {
        unsigned char cmd = 0;
        rd(in, &cmd, 1);
        if (cmd == 0) break;
        if (buf) (void)hipFree(buf);
        (void)hipMalloc(&buf, kSize);
        (void)hipMemset(buf, fill, kSize);
        (void)hipDeviceSynchronize();
        reply r{};
        (void)hipIpcGetMemHandle(&r.h, buf);
        r.va = buf;
        wr(out, &r, sizeof(r));
    }
    if (buf) (void)hipFree(buf);
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 20;
    int to[2][2], from[2][2];
    pid_t kids[2];
    const unsigned char fills[2] = {0x11, 0x22};
    for (int k = 0; k < 2; ++k) {
        if (pipe(to[k]) || pipe(from[k])) return 2;
        kids[k] = fork();
        if (kids[k] == 0) {
            exporter(to[k][0], from[k][1], fills[k]);
            _exit(0);
        }
    }
    for (int keep = 0; keep < 2; ++keep) {
        int same_va = 0, wrong = 0, errs = 0;
        void *prev[2] = {nullptr, nullptr};
        for (int r = 0; r < rounds; ++r) {
            reply rep[2];
            for (int k = 0; k < 2; ++k) {
                unsigned char go = 1;
                wr(to[k][1], &go, 1);
                rd(from[k][0], &rep[k], sizeof(reply));
            }
            same_va += rep[0].va == rep[1].va;
            void *m[2] = {nullptr, nullptr};
            for (int k = 0; k < 2; ++k) {
                if (hipIpcOpenMemHandle(&m[k], rep[k].h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                    ++errs;
                    m[k] = nullptr;
                    continue;
                }
                unsigned char b = 0;
                (void)hipMemcpy(&b, (char *)m[k] + kSize / 2, 1, hipMemcpyDeviceToHost);
                if (b != fills[k]) ++wrong;
            }
            for (int k = 0; k < 2; ++k) {
                if (keep) {
                    if (prev[k]) (void)hipIpcCloseMemHandle(prev[k]);
                    prev[k] = m[k];
                } else if (m[k]) {
                    (void)hipIpcCloseMemHandle(m[k]);
                }
            }
        }
        for (int k = 0; k < 2; ++k)
            if (prev[k]) (void)hipIpcCloseMemHandle(prev[k]);
        printf("scenario %-5s rounds %d: exporters at the same address %d, wrong bytes %d, open "
               "errors %d\n", keep ? "keep" : "close", rounds, same_va, wrong, errs);
        fflush(stdout);
    }
    for (int k = 0; k < 2; ++k) {
        unsigned char q = 0;
        wr(to[k][1], &q, 1);
        waitpid(kids[k], nullptr, 0);
    }
    return 0;
}
