"""Host->device bandwidth probe: pinned int16 buffer of one 256-slot batch (92 MB), one copy vs
chunked copies on 1/2/4 streams."""
import time
import torch

if __name__ == "__main__":
    n = 256 * 180000
    h = torch.empty(n, dtype=torch.int16).pin_memory()
    d = torch.empty(n, dtype=torch.int16, device="cuda")
    for ns in (1, 2, 4):
        ss = [torch.cuda.Stream() for _ in range(ns)]
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for it in range(10):
                ch = n // ns
                for k, s in enumerate(ss):
                    with torch.cuda.stream(s):
                        d[k * ch:(k + 1) * ch].copy_(h[k * ch:(k + 1) * ch], non_blocking=True)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
        print(f"streams {ns}: {dt * 1e3:.2f} ms per 92 MB batch, {2 * n / dt / 1e9:.1f} GB/s", flush=True)
