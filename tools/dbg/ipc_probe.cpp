// IPC timing probe: rank 0 allocates `mb` MiB, exports a handle to a file; rank 1 opens it.
// usage: ipc_probe <rank> <mb> <file>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <unistd.h>
#include <fcntl.h>
#include <sys/mman.h>
static double now() { timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }
int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int rank = atoi(argv[1]);
    const size_t mb = strtoull(argv[2], nullptr, 10);
    const char* f = argv[3];
    double t0 = now();
    if (hipSetDevice(0) != hipSuccess) return 2;
    printf("r%d init %.3f s\n", rank, now() - t0);
    if (argc > 4 && argv[4][0] == 'r') {                 // register a shared mapping first
        int fd = shm_open("/ipc_probe_shm", O_CREAT | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, 1 << 20) != 0) return 4;
        void* m = mmap(nullptr, 1 << 20, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        hipError_t e = hipHostRegister(m, 1 << 20, hipHostRegisterMapped);
        printf("r%d shm register rc %d\n", rank, int(e));
    }
    if (argc > 5) {                                       // several allocations first
        void* q = nullptr;
        for (int i = 0; i < atoi(argv[5]); i++) (void)hipMalloc(&q, size_t(64) << 20);
        printf("r%d %d extra allocations\n", rank, atoi(argv[5]));
    }
    if (rank == 0) {
        void* p = nullptr;
        t0 = now();
        hipError_t e = hipMalloc(&p, mb << 20);
        printf("r0 malloc %zu MiB rc %d %.3f s\n", mb, int(e), now() - t0);
        hipIpcMemHandle_t h;
        t0 = now();
        e = hipIpcGetMemHandle(&h, p);
        printf("r0 get handle rc %d %.3f s\n", int(e), now() - t0);
        FILE* o = fopen(f, "wb"); fwrite(&h, sizeof h, 1, o); fclose(o);
        char done[256]; snprintf(done, sizeof done, "%s.done", f);
        for (int i = 0; i < 600 && access(done, F_OK) != 0; i++) usleep(100000);
        printf("r0 peer done\n");
        (void)hipFree(p);
    } else {
        for (int i = 0; i < 600 && access(f, F_OK) != 0; i++) usleep(100000);
        usleep(200000);
        hipIpcMemHandle_t h;
        FILE* in = fopen(f, "rb"); if (!in || fread(&h, sizeof h, 1, in) != 1) return 3; fclose(in);
        void* p = nullptr;
        t0 = now();
        hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        printf("r1 open rc %d %.3f s ptr %p\n", int(e), now() - t0, p);
        t0 = now();
        if (e == hipSuccess) e = hipMemset(p, 1, 1 << 20);
        printf("r1 memset rc %d %.3f s\n", int(e), now() - t0);
        t0 = now();
        if (p) e = hipIpcCloseMemHandle(p);
        printf("r1 close rc %d %.3f s\n", int(e), now() - t0);
        char done[256]; snprintf(done, sizeof done, "%s.done", f);
        FILE* d = fopen(done, "w"); fclose(d);
    }
    return 0;
}
