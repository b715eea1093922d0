// Host-registration probe, round 5: what do the HSA runtime's pointer table (hsa_amd_pointer_info:
// the locked-range records ROCr keeps for hsa_amd_memory_lock, under HIP's own map) and HIP's
// pageable-copy path do around the host tests' pattern? No kernel runs; every DMA reads or writes
// memory that is registered or freshly allocated at that moment, and the one step that copies
// from a re-mapped, previously registered address runs last.
// Build: hipcc -O1 -o tools/hostreg_probe2 tools/hostreg_probe2.cpp -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

static const char* ptype(hsa_amd_pointer_type_t t) {
    switch (int(t)) {
    case HSA_EXT_POINTER_TYPE_UNKNOWN: return "unknown";
    case HSA_EXT_POINTER_TYPE_HSA: return "hsa";
    case HSA_EXT_POINTER_TYPE_LOCKED: return "locked";
    case HSA_EXT_POINTER_TYPE_GRAPHICS: return "graphics";
    case HSA_EXT_POINTER_TYPE_IPC: return "ipc";
    default: return "other";
    }
}

static void info(const char* what, const void* p) {
    hsa_amd_pointer_info_t in;
    memset(&in, 0, sizeof in);
    in.size = sizeof in;
    hsa_status_t s = hsa_amd_pointer_info(const_cast<void*>(p), &in, nullptr, nullptr, nullptr);
    printf("  %-40s p=%p st=%d type=%-8s host=%p agent=%p bytes=%zu\n", what, p, int(s), ptype(in.type),
           in.hostBaseAddress, in.agentBaseAddress, size_t(in.sizeInBytes));
}

static const uintptr_t kPage = 4096;
static const void* page_of(const void* p) { return reinterpret_cast<const void*>(uintptr_t(p) & ~(kPage - 1)); }

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const char* only = argc > 1 ? argv[1] : "12345";
    auto want = [&](char c) { return strchr(only, c) != nullptr; };
    if (hipSetDevice(0) != hipSuccess || hsa_init() != HSA_STATUS_SUCCESS) return 2;
    void* dev = nullptr;
    const size_t dev_bytes = 256u << 20;
    if (hipMalloc(&dev, dev_bytes) != hipSuccess) return 3;

    // 1: which path a pageable H2D copy takes by size (run with AMD_LOG_LEVEL=3 and read the
    //    "Pinned resource" / "Staging resource" lines), and whether the source is left locked.
    if (want('1')) {
        printf("1: pageable copies by size\n");
        const size_t sizes[] = {256u << 10, 1u << 20, 1200000, 4u << 20, 16u << 20, 64u << 20, 200u << 20};
        for (size_t sz : sizes) {
            char* h = static_cast<char*>(malloc(sz));
            memset(h, 7, sz);
            fprintf(stderr, "=== copy %zu bytes ===\n", sz);
            hipError_t e = hipMemcpy(dev, h, sz, hipMemcpyHostToDevice);
            char tag[64];
            snprintf(tag, sizeof tag, "src of %zu-byte copy (rc %d)", sz, int(e));
            info(tag, h);
            info("  its middle", h + sz / 2);
            free(h);
        }
    }

    char* arena = static_cast<char*>(aligned_alloc(kPage, 64u << 20));
    memset(arena, 1, 64u << 20);
    const size_t l1 = 1582736, l2 = 524308;

    // 2: two registrations sharing a page, unregistered one at a time
    if (want('2')) {
        printf("2: two registrations on a shared page\n");
        char* b1 = arena + 100;
        char* b2 = b1 + l1 + 16;
        printf("  register b1 %d b2 %d\n", int(hipHostRegister(b1, l1, hipHostRegisterDefault)),
               int(hipHostRegister(b2, l2, hipHostRegisterDefault)));
        info("b1", b1);
        info("b2", b2);
        info("shared page", page_of(b2));
        info("b2 last byte", b2 + l2 - 1);
        printf("  unregister b1 %d\n", int(hipHostUnregister(b1)));
        info("b1 after b1 unregistered", b1);
        info("shared page after b1 unregistered", page_of(b2));
        info("b2 after b1 unregistered", b2);
        info("b2 +page after b1 unregistered", b2 + kPage);
        printf("  unregister b2 %d\n", int(hipHostUnregister(b2)));
        info("b2 after both", b2);
        info("shared page after both", page_of(b2));
    }

    // 3: a registration and a pageable copy from a neighbour on its last page (the runtime's own
    //    pinning of pageable memory next to a registration)
    if (want('3')) {
        printf("3: pageable copy from a neighbour of a registration\n");
        char* r = arena + (8u << 20) + 100;
        char* nb = r + l1 + 16;                          // starts on r's last page, never registered
        const size_t ln = 1200000;
        printf("  register r %d\n", int(hipHostRegister(r, l1, hipHostRegisterDefault)));
        fprintf(stderr, "=== neighbour copy ===\n");
        printf("  pageable copy from neighbour %d\n", int(hipMemcpy(dev, nb, ln, hipMemcpyHostToDevice)));
        info("r after neighbour copy", r);
        info("neighbour after its copy", nb);
        info("neighbour +page", nb + kPage);
        printf("  unregister r %d\n", int(hipHostUnregister(r)));
        info("r after unregister", r);
        info("neighbour after r unregistered", nb);
    }

    // 4: register, DMA into it, unregister, munmap, map again at the same address; what the
    //    runtime's table holds for the new mapping (no copy yet)
    const size_t lm = 8u << 20;
    char* m = nullptr;
    if (want('4') || want('5')) {
        m = static_cast<char*>(mmap(nullptr, lm, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
        if (m == MAP_FAILED) return 4;
        memset(m, 3, lm);
        char* mr = m + 100;
        printf("4: register, copy, unregister, munmap, remap at %p\n", (void*)m);
        printf("  register %d\n", int(hipHostRegister(mr, lm - 200, hipHostRegisterDefault)));
        printf("  D2H into registered %d\n", int(hipMemcpy(mr, dev, lm - 200, hipMemcpyDeviceToHost)));
        printf("  H2D from registered %d\n", int(hipMemcpy(dev, mr, lm - 200, hipMemcpyHostToDevice)));
        printf("  unregister %d\n", int(hipHostUnregister(mr)));
        info("after unregister", mr);
        printf("  munmap %d\n", munmap(m, lm));
        char* m2 = static_cast<char*>(mmap(m, lm, PROT_READ | PROT_WRITE,
                                           MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED_NOREPLACE, -1, 0));
        printf("  remap %p (same: %d)\n", (void*)m2, int(m2 == m));
        if (m2 == MAP_FAILED) return 5;
        memset(m2, 4, lm);
        info("remapped start", m2 + 100);
        info("remapped middle", m2 + lm / 2);
        m = m2;
    }
    // 5 (last): a pageable copy from the re-mapped, once-registered address range
    if (want('5')) {
        printf("5: pageable copy from the re-mapped range\n");
        fprintf(stderr, "=== remapped copy ===\n");
        hipError_t e = hipMemcpy(dev, m + 100, 1200000, hipMemcpyHostToDevice);
        printf("  copy %d\n", int(e));
        e = hipMemcpy(dev, m + 100, lm - 200, hipMemcpyHostToDevice);
        printf("  copy whole %d\n", int(e));
        printf("  sync %d\n", int(hipDeviceSynchronize()));
        info("remapped after copies", m + 100);
    }
    printf("done\n");
    return 0;
}
