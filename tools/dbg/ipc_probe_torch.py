"""IPC export/open between two torch-initialised processes (ctypes on libamdhip64), by size."""
import ctypes
import os
import subprocess
import sys
import time

if len(sys.argv) > 1:
    rank, mb, f = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    import torch
    torch.zeros(1, device="cuda")                          # torch's HIP context
    hip = ctypes.CDLL("libamdhip64.so")
    p = ctypes.c_void_p()
    if rank == 0:
        t0 = time.time()
        rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(mb << 20))
        h = (ctypes.c_char * 64)()
        rc2 = hip.hipIpcGetMemHandle(h, p)
        open(f, "wb").write(bytes(h))
        print(f"r0 {mb} MiB malloc {rc} handle {rc2} {time.time() - t0:.3f}s", flush=True)
        for _ in range(300):
            if os.path.exists(f + ".done"):
                break
            time.sleep(0.1)
    else:
        for _ in range(300):
            if os.path.exists(f):
                break
            time.sleep(0.1)
        time.sleep(0.3)
        h = (ctypes.c_char * 64).from_buffer_copy(open(f, "rb").read())
        t0 = time.time()
        print(f"r1 {mb} MiB opening", flush=True)
        rc = hip.hipIpcOpenMemHandle(ctypes.byref(p), h, ctypes.c_uint(1))
        print(f"r1 {mb} MiB open {rc} {time.time() - t0:.3f}s", flush=True)
        hip.hipIpcCloseMemHandle(p)
        open(f + ".done", "w").close()
    sys.exit(0)

for mb in (9, 600, 1200, 2416):
    f = f"/tmp/ipct_{mb}"
    for x in (f, f + ".done"):
        if os.path.exists(x):
            os.remove(x)
    ps = [subprocess.Popen([sys.executable, "-u", __file__, str(r), str(mb), f]) for r in range(2)]
    try:
        rcs = [p.wait(timeout=40) for p in ps]
    except subprocess.TimeoutExpired:
        for p in ps:
            p.kill()
        rcs = "timeout"
    print(f"size {mb} MiB: {rcs}", flush=True)
