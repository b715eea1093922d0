// Host-registration probe (no kernel, no copy touches a stale range): what does the HIP runtime
// report for a host range after hipHostUnregister, when two registrations share a page (the
// round-3 host tests registered two numpy arrays that glibc may place on one page) and when a
// registration stands alone? Build: hipcc -O1 -o tools/hostreg_probe tools/hostreg_probe.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <malloc.h>

static const char* mt(hipMemoryType t) {
    switch (t) {
    case hipMemoryTypeHost: return "host(registered)";
    case hipMemoryTypeDevice: return "device";
    case hipMemoryTypeUnified: return "unified";
    default: return "unregistered";
    }
}

static void show(const char* what, void* p) {
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof a);
    hipError_t e = hipPointerGetAttributes(&a, p);
    unsigned int flags = 0;
    hipError_t ef = hipHostGetFlags(&flags, p);
    void* dp = nullptr;
    hipError_t ed = hipHostGetDevicePointer(&dp, p, 0);
    printf("  %-34s attr=%-3d type=%-16s hostPtr=%p devPtr=%p | getFlags=%d | getDevPtr=%d %p\n", what, int(e),
           e == hipSuccess ? mt(a.type) : "-", a.hostPointer, a.devicePointer, int(ef), int(ed), dp);
    (void)hipGetLastError();
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const char* only = argc > 1 ? argv[1] : "ABCDE";
    auto want = [&](char c) { return strchr(only, c) != nullptr; };
    const size_t page = 4096;
    char* arena = static_cast<char*>(aligned_alloc(page, 64 << 20));
    memset(arena, 1, 64 << 20);

    printf("arena %p\n", (void*)arena);
    // A: one registration, unregistered
    if (want('A')) {
    printf("A: single range\n");
    char* a = arena + 100;
    size_t la = 1582736;
    printf("  register %d\n", int(hipHostRegister(a, la, hipHostRegisterDefault)));
    show("a (registered)", a);
    printf("  unregister %d\n", int(hipHostUnregister(a)));
    show("a after unregister", a);
    show("a+page after unregister", a + page);
    }

    // B: two ranges sharing a page (b2 starts inside b1's last page)
    const size_t l1 = 1582736, l2 = 791368;
    if (want('B')) {
    printf("B: two ranges on a shared page\n");
    char* b1 = arena + (8 << 20) + 100;
    char* b2 = b1 + l1 + 16;
    printf("  register b1 %d\n", int(hipHostRegister(b1, l1, hipHostRegisterDefault)));
    printf("  register b2 %d\n", int(hipHostRegister(b2, l2, hipHostRegisterDefault)));
    show("b1", b1);
    show("b2", b2);
    printf("  unregister b1 %d\n", int(hipHostUnregister(b1)));
    printf("  unregister b2 %d\n", int(hipHostUnregister(b2)));
    show("b1 after unregister", b1);
    show("b1 mid after unregister", b1 + l1 / 2);
    show("b2 after unregister", b2);
    show("b2 mid after unregister", b2 + l2 / 2);
    show("shared page after unregister", (char*)((uintptr_t)(b2) & ~(page - 1)));
    }

    // C: B in the other unregister order
    if (want('C')) {
    printf("C: shared page, unregister b2 first\n");
    char* c1 = arena + (16 << 20) + 100;
    char* c2 = c1 + l1 + 16;
    printf("  register c1 %d c2 %d\n", int(hipHostRegister(c1, l1, hipHostRegisterDefault)),
           int(hipHostRegister(c2, l2, hipHostRegisterDefault)));
    printf("  unregister c2 %d c1 %d\n", int(hipHostUnregister(c2)), int(hipHostUnregister(c1)));
    show("c1 after unregister", c1);
    show("c2 after unregister", c2);
    }

    // D: the same range registered twice
    if (want('D')) {
    printf("D: same range twice\n");
    char* d = arena + (24 << 20);
    const size_t la = 1582736;
    printf("  register %d, again %d\n", int(hipHostRegister(d, la, hipHostRegisterDefault)),
           int(hipHostRegister(d, la, hipHostRegisterDefault)));
    printf("  unregister %d, again %d\n", int(hipHostUnregister(d)), int(hipHostUnregister(d)));
    show("d after unregister x2", d);
    }

    // E: a pointer inside a registered range that is not its start
    if (want('E')) {
    printf("E: unregister by an interior pointer\n");
    char* e = arena + (32 << 20) + 64;
    const size_t la = 1582736;
    printf("  register %d, unregister(e+4096) %d, unregister(e) %d\n",
           int(hipHostRegister(e, la, hipHostRegisterDefault)), int(hipHostUnregister(e + 4096)),
           int(hipHostUnregister(e)));
    show("e after unregister", e);
    }
    // F / G: the host tests' pattern -- two buffers registered, unregistered, freed; the next
    // allocations of the same sizes (often the same addresses) are never registered: what does
    // the runtime report for them? G puts the buffers on the heap (sharing pages), as glibc does
    // once its mmap threshold has grown.
    for (char sc : {'F', 'G'}) {
        if (!want(sc)) continue;
        if (sc == 'G') mallopt(M_MMAP_THRESHOLD, 64 << 20);
        printf("%c: register, unregister, free, reallocate (%s)\n", sc, sc == 'F' ? "malloc default" : "heap");
        char* x1 = static_cast<char*>(malloc(l1));
        char* x2 = static_cast<char*>(malloc(l2));
        memset(x1, 2, l1);
        memset(x2, 3, l2);
        printf("  x1 %p x2 %p\n", (void*)x1, (void*)x2);
        printf("  register x1 %d x2 %d\n", int(hipHostRegister(x1, l1, hipHostRegisterDefault)),
               int(hipHostRegister(x2, l2, hipHostRegisterDefault)));
        printf("  unregister x1 %d x2 %d\n", int(hipHostUnregister(x1)), int(hipHostUnregister(x2)));
        free(x2);
        free(x1);
        char* y1 = static_cast<char*>(malloc(l1));
        char* y2 = static_cast<char*>(malloc(l2));
        memset(y1, 4, l1);
        memset(y2, 5, l2);
        printf("  y1 %p y2 %p (never registered)\n", (void*)y1, (void*)y2);
        show("y1", y1);
        show("y1 mid", y1 + l1 / 2);
        show("y2", y2);
        free(y1);
        free(y2);
    }
    return 0;
}
