// Diagnostic for the IPC mapping-aliasing failure (VERDICT r01
// "weak" 2).  Two processes on one device, forked per scenario from a parent
// that never touches HIP: the importer drives a script, the exporter
// allocates / fills / frees / exports on command.  For every open it prints
// the address, whether the exporter reused a virtual address, the buffer
// ids, and whether the bytes seen through the mapping are the new
// allocation's (else STALE).
#include <hip/hip_runtime.h>
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

struct cmd {
    int op;  // 0 alloc, 1 free, 2 export, 3 quit
    int slot;
    size_t bytes;
    int fill;
};
struct reply {
    int rc;
    void *ptr;
    unsigned long long id;
    hipIpcMemHandle_t h;
};

static int c2e[2], e2c[2];

static void wr(int fd, const void *p, size_t n) {
    if (write(fd, p, n) != (ssize_t)n) _exit(4);
}
static void rd(int fd, void *p, size_t n) {
    if (read(fd, p, n) != (ssize_t)n) _exit(5);
}

static unsigned long long buf_id(void *p) {
    unsigned long long id = 0;
    if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return id;
}

static void exporter() {
    close(c2e[1]);
    close(e2c[0]);
    if (hipSetDevice(0) != hipSuccess) _exit(6);
    void *slot[16] = {};
    for (;;) {
        cmd c;
        rd(c2e[0], &c, sizeof(c));
        reply r{};
        if (c.op == 3) break;
        if (c.op == 0) {
            hipError_t e = hipMalloc(&slot[c.slot], c.bytes);
            if (e == hipSuccess) e = hipMemset(slot[c.slot], c.fill, c.bytes);
            if (e == hipSuccess) e = hipDeviceSynchronize();
            r.rc = e;
            r.ptr = slot[c.slot];
            r.id = e == hipSuccess ? buf_id(slot[c.slot]) : 0;
        } else if (c.op == 1) {
            r.rc = hipFree(slot[c.slot]);
            r.ptr = slot[c.slot];
            slot[c.slot] = nullptr;
        } else if (c.op == 2) {
            r.rc = hipIpcGetMemHandle(&r.h, slot[c.slot]);
            if (r.rc != hipSuccess) (void)hipGetLastError();
            r.ptr = slot[c.slot];
            r.id = buf_id(slot[c.slot]);
        }
        wr(e2c[1], &r, sizeof(r));
    }
    _exit(0);
}

// ---- importer side
static reply ex(int op, int s, size_t bytes = 0, int fill = 0) {
    cmd c{op, s, bytes, fill};
    wr(c2e[1], &c, sizeof(c));
    reply r;
    rd(e2c[0], &r, sizeof(r));
    return r;
}
static unsigned long long hh(const hipIpcMemHandle_t &h) {  // FNV-1a of the handle bytes
    unsigned long long x = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(h); ++i) x = (x ^ (unsigned char)h.reserved[i]) * 1099511628211ull;
    return x;
}

static void *exp_ptr[16];
static int exp_fill[16];
static reply H[16];

static void alloc(int s, size_t mib, int fill) {
    reply r = ex(0, s, mib << 20, fill);
    bool reused = false;
    for (int i = 0; i < 16; ++i) reused = reused || (i != s && exp_ptr[i] == r.ptr);
    printf("  E alloc  s%d %4zu MiB -> %p id %llu rc %d%s\n", s, mib, r.ptr, r.id, r.rc,
           reused ? "  (REUSES an earlier VA)" : "");
    exp_ptr[s] = r.ptr;
    exp_fill[s] = fill;
}
static void efree(int s) {
    reply r = ex(1, s);
    printf("  E free   s%d -> rc %d\n", s, r.rc);
}
static bool eexport(int s) {
    reply r = ex(2, s);
    H[s] = r;
    printf("  E export s%d (%p id %llu) -> rc %d %s handle %016llx\n", s, r.ptr, r.id, r.rc,
           r.rc ? hipGetErrorString((hipError_t)r.rc) : "", hh(r.h));
    return r.rc == 0;
}
static void *iopen(int s) {
    void *m = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&m, H[s].h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        printf("  I open   s%d -> %s\n", s, hipGetErrorString(e));
        return nullptr;
    }
    unsigned char v = 0;
    e = hipMemcpy(&v, (char *)m + 4096, 1, hipMemcpyDeviceToHost);
    printf("  I open   s%d -> %p byte 0x%02x expected 0x%02x%s\n", s, m, v, exp_fill[s],
           (e == hipSuccess && v == exp_fill[s]) ? "" : "  STALE/ALIAS");
    return m;
}
static void iclose(void *m, const char *what) {
    if (!m) return;
    hipError_t e = hipIpcCloseMemHandle(m);
    printf("  I close  %s -> %d\n", what, e);
}

static void scenario(int k) {
    if (hipSetDevice(0) != hipSuccess) _exit(6);
    void *m0 = nullptr, *m1 = nullptr, *m2 = nullptr;
    switch (k) {
    case 1:  // stale import kept open; exporter frees, reallocates same size
        printf("S1: import kept open, exporter free -> alloc same size -> export -> open\n");
        alloc(0, 32, 0x10); eexport(0); m0 = iopen(0);
        efree(0); alloc(1, 32, 0x11);
        if (eexport(1)) m1 = iopen(1);
        alloc(2, 64, 0x12); efree(1);
        if (eexport(2)) m2 = iopen(2);
        iclose(m0, "m0"); iclose(m1, "m1"); iclose(m2, "m2");
        break;
    case 2:  // import closed before the free
        printf("S2: import closed, exporter free -> alloc same size -> export -> open\n");
        alloc(0, 32, 0x20); eexport(0); m0 = iopen(0); iclose(m0, "m0");
        efree(0); alloc(1, 32, 0x21);
        if (eexport(1)) m1 = iopen(1);
        iclose(m1, "m1");
        break;
    case 3:  // never imported
        printf("S3: exported, never imported, free -> alloc same size -> export -> open\n");
        alloc(0, 32, 0x30); eexport(0);
        efree(0); alloc(1, 32, 0x31);
        if (eexport(1)) m1 = iopen(1);
        iclose(m1, "m1");
        break;
    case 4:  // landing growth: close, alloc new, export, free old, open
        printf("S4: landing growth x3 (importer closes first; alloc new, export, free old)\n");
        alloc(0, 32, 0x40); eexport(0); m0 = iopen(0);
        for (int g = 1; g <= 3; ++g) {
            iclose(m0, "old landing");
            alloc(g, (size_t)32 << g, 0x40 + g);
            bool ok = eexport(g);
            efree(g - 1);
            m0 = ok ? iopen(g) : nullptr;
        }
        iclose(m0, "last");
        break;
    case 5:  // a user buffer stays in the importer's cache after the exporter frees it;
             // then a landing-style allocation of the same size
        printf("S5: user import cached open, exporter frees it, landing alloc same size\n");
        alloc(0, 32, 0x50); eexport(0); m0 = iopen(0);   // cached user-buffer import
        alloc(1, 32, 0x51); eexport(1); m1 = iopen(1);   // old landing
        efree(0);                                        // user frees its buffer
        iclose(m1, "old landing");                       // growth: close landing mapping
        alloc(2, 32, 0x52);                              // new landing (may reuse s0's VA)
        if (eexport(2)) m2 = iopen(2);
        efree(1);
        iclose(m2, "new landing"); iclose(m0, "stale user import");
        break;
    case 6:  // as S5, then the stale import is closed and the landing re-exported
        printf("S6: S5 then close the stale import and retry export/open of a fresh alloc\n");
        alloc(0, 32, 0x60); eexport(0); m0 = iopen(0);
        efree(0);
        alloc(1, 32, 0x61);
        if (eexport(1)) { m1 = iopen(1); iclose(m1, "m1"); }
        iclose(m0, "stale user import");
        alloc(2, 32, 0x62);
        if (eexport(2)) { m2 = iopen(2); iclose(m2, "m2"); }
        efree(1);
        alloc(3, 32, 0x63);
        if (eexport(3)) { void *m3 = iopen(3); iclose(m3, "m3"); }
        break;
    case 7:  // importer keeps the old mapping; a larger allocation takes the freed range
        printf("S7: import kept open, free 16 MiB, alloc 18 MiB (same start), export\n");
        alloc(0, 16, 0x70); eexport(0); m0 = iopen(0);
        efree(0); alloc(1, 18, 0x71);
        if (eexport(1)) { m1 = iopen(1); iclose(m1, "m1"); }
        iclose(m0, "stale m0");
        if (eexport(1)) { m1 = iopen(1); iclose(m1, "m1 after the stale close"); }
        break;
    case 8:  // as S7, importer closed before the free
        printf("S8: import closed, free 16 MiB, alloc 18 MiB, export\n");
        alloc(0, 16, 0x80); eexport(0); m0 = iopen(0); iclose(m0, "m0");
        efree(0); alloc(1, 18, 0x81);
        if (eexport(1)) { m1 = iopen(1); iclose(m1, "m1"); }
        break;
    case 9:  // a smaller allocation inside the freed, still-imported range
        printf("S9: import kept open, free 16 MiB, alloc 8 MiB, export\n");
        alloc(0, 16, 0x90); eexport(0); m0 = iopen(0);
        efree(0); alloc(1, 8, 0x91);
        if (eexport(1)) { m1 = iopen(1); iclose(m1, "m1"); }
        iclose(m0, "stale m0");
        break;
    case 10:  // two freed, still-imported neighbours, one allocation spanning both
        printf("S10: two imports kept open, both freed, alloc spanning both, export\n");
        alloc(0, 16, 0xa0); eexport(0); m0 = iopen(0);
        alloc(1, 16, 0xa1); eexport(1); m1 = iopen(1);
        efree(0); efree(1); alloc(2, 32, 0xa2);
        if (eexport(2)) { m2 = iopen(2); iclose(m2, "m2"); }
        iclose(m0, "stale m0"); iclose(m1, "stale m1");
        if (eexport(2)) { m2 = iopen(2); iclose(m2, "m2 after the stale closes"); }
        break;
    case 13: {  // the collective pattern: mapping open, peer frees + reallocates the same
                // size (same handle bytes?), importer closes the old mapping and opens the
                // new handle at once; 30 rounds, contents checked every time
        printf("S13: 30 x (open A; free A; alloc B same size; export B; close A; open B)\n");
        alloc(0, 16, 0xd0); eexport(0); m0 = iopen(0);
        for (int rnd = 1; rnd <= 30; ++rnd) {
            const int a = (rnd - 1) & 1, b = rnd & 1;
            unsigned long long ha = hh(H[a].h);
            efree(a);
            alloc(b, 16, 0xd0 + rnd);
            eexport(b);
            printf("  round %d: handle %s\n", rnd, hh(H[b].h) == ha ? "REUSED" : "new");
            iclose(m0, "old");
            m0 = iopen(b);
        }
        iclose(m0, "last");
        break;
    }
    case 11:  // the IMPORTER closes a peer mapping, then allocates and exports its own buffer
    case 12: {  // as 11, the mapping still open while it allocates
        printf("S%d: importer %s a peer mapping, then allocates + exports its own 16 MiB\n", k,
               k == 11 ? "opens and closes" : "keeps open");
        alloc(0, 16, 0xb0); eexport(0); m0 = iopen(0);
        if (k == 11) iclose(m0, "m0");
        for (int rep = 0; rep < 3; ++rep) {
            void *own = nullptr;
            hipError_t e = hipMalloc(&own, (size_t)(16 + 2 * rep) << 20);
            void *base = nullptr;
            size_t range = 0;
            hipError_t e2 = hipMemGetAddressRange((hipDeviceptr_t *)&base, &range, (hipDeviceptr_t)own);
            hipIpcMemHandle_t h;
            hipError_t e3 = hipIpcGetMemHandle(&h, base ? base : own);
            printf("  I own alloc %p (rc %d) range %p + %zu (rc %d)%s -> export rc %d %s\n", own, e,
                   base, range, e2, own == m0 ? "  (the closed mapping's address)" : "", e3,
                   e3 ? hipGetErrorString(e3) : "");
            (void)hipGetLastError();
            (void)hipFree(own);
        }
        if (k == 12) iclose(m0, "m0");
        break;
    }
    }
    cmd q{3, 0, 0, 0};  // quit: no reply
    wr(c2e[1], &q, sizeof(q));
    fflush(stdout);
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    int k0 = argc > 1 ? atoi(argv[1]) : 1;
    for (int k = k0; k <= 13; ++k) {
        if (pipe(c2e) || pipe(e2c)) return 1;
        fflush(stdout);
        pid_t e = fork();
        if (e == 0) { alarm(20); exporter(); }
        pid_t i = fork();
        if (i == 0) {
            alarm(20);
            close(c2e[0]);
            close(e2c[1]);
            scenario(k);
            _exit(0);
        }
        close(c2e[0]); close(c2e[1]); close(e2c[0]); close(e2c[1]);
        int st1 = 0, st2 = 0;
        waitpid(i, &st1, 0);
        waitpid(e, &st2, 0);
        printf("  (importer status %d, exporter status %d)\n\n", st1, st2);
        fflush(stdout);
    }
    return 0;
}
