import torch, time
dev = torch.device("cuda:0")
n = 4 << 30
buf = torch.empty(n, dtype=torch.uint8, device=dev)
for name, fn in [("memset0", lambda: buf.zero_()), ("fill_ff", lambda: buf.fill_(255))]:
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10): fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    print(name, "%.3f ms  %.2f TB/s" % (dt * 1e3, n / dt / 1e12))
v = buf.view(torch.int64)
import ctypes
