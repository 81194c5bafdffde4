// Does a THIRD process's open mapping of a freed allocation leak into a new
// export at the same address?  Three processes, forked before any HIP call:
//   E (exporter)  allocates A, fills it with 0xAA.., exports hA;
//   H (holder)    opens hA and keeps it open (scenario "held") or closes it
//                 at once (scenario "closed");
//   I (importer)  opens hA, checks it, closes it (scenario "I held": keeps
//                 it open while it opens hB);
// then E frees A, allocates B of the same size (it usually gets A's address),
// fills it with 0xBB.., exports hB (different handle bytes), and I opens hB
// and reports what it reads.  0xAA through hB = the runtime served the freed
// allocation that H still holds.  Rounds repeat with fresh buffers.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

struct msg {
    hipIpcMemHandle_t h;
    int cmd;  // 1 open+check(expect) 2 close 3 quit 4 open+hold
    unsigned char expect;
};

static size_t kSize = 8u << 20;   // A's size
static size_t kSizeB = 8u << 20;  // B's size (argv[2] MiB*1000: a smaller B inside A's old range)

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

// a peer process: obeys commands, answers with one byte read from the mapping
static void peer(int in, int out) {
    void *held = nullptr;
    for (;;) {
        msg m;
        rd(in, &m, sizeof(m));
        unsigned char ans = 0;
        if (m.cmd == 3) break;
        if (m.cmd == 2) {
            if (held) (void)hipIpcCloseMemHandle(held);
            held = nullptr;
        } else {
            void *p = nullptr;
            if (hipIpcOpenMemHandle(&p, m.h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                ans = 0xEE;
            } else {
                (void)hipMemcpy(&ans, (char *)p + 4096, 1, hipMemcpyDeviceToHost);
                if (m.cmd == 4) held = p;
                else (void)hipIpcCloseMemHandle(p);
            }
        }
        wr(out, &ans, 1);
    }
    if (held) (void)hipIpcCloseMemHandle(held);
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 20;
    if (argc > 2) kSizeB = (size_t)atol(argv[2]);
    if (argc > 3) kSize = (size_t)atol(argv[3]);
    int to[2][2], from[2][2];
    pid_t kids[2];
    for (int k = 0; k < 2; ++k) {
        if (pipe(to[k]) || pipe(from[k])) return 2;
        kids[k] = fork();
        if (kids[k] == 0) {
            peer(to[k][0], from[k][1]);
            _exit(0);
        }
    }
    auto ask = [&](int k, const hipIpcMemHandle_t &h, int cmd) {
        msg m{};
        m.h = h;
        m.cmd = cmd;
        wr(to[k][1], &m, sizeof(m));
        unsigned char a = 0;
        rd(from[k][0], &a, 1);
        return a;
    };
    const int H = 0, I = 1;
    const char *names[3] = {"closed", "H held", "I held"};
    for (int held = 0; held < 3; ++held) {
        int same_addr = 0, stale = 0, errs = 0;
        for (int r = 0; r < rounds; ++r) {
            void *a = nullptr, *b = nullptr;
            hipIpcMemHandle_t ha, hb;
            (void)hipMalloc(&a, kSize);
            (void)hipMemset(a, 0xAA, kSize);
            (void)hipDeviceSynchronize();
            (void)hipIpcGetMemHandle(&ha, a);
            ask(H, ha, held == 1 ? 4 : 1);
            if (ask(I, ha, held == 2 ? 4 : 1) != 0xAA) ++errs;
            (void)hipFree(a);
            (void)hipMalloc(&b, kSizeB);
            (void)hipMemset(b, 0xBB, kSizeB);
            (void)hipDeviceSynchronize();
            (void)hipIpcGetMemHandle(&hb, b);
            same_addr += (char *)b >= (char *)a && (char *)b < (char *)a + kSize;
            const unsigned char seen = ask(I, hb, 1);
            if (seen == 0xAA) ++stale;
            else if (seen != 0xBB) ++errs;
            if (held == 1) ask(H, ha, 2);
            if (held == 2) ask(I, ha, 2);
            (void)hipFree(b);
        }
        printf("A %zu B %zu scenario %-6s rounds %d: B inside A's old range %d, importer saw A's bytes through hB %d, "
               "other errors %d\n", kSize, kSizeB, names[held], rounds, same_addr, stale, errs);
        fflush(stdout);
    }
    for (int k = 0; k < 2; ++k) {
        msg m{};
        m.cmd = 3;
        wr(to[k][1], &m, sizeof(m));
        waitpid(kids[k], nullptr, 0);
    }
    return 0;
}
