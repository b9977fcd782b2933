"""Lab probe: which torch streams share a hardware queue.  Two spin kernels on two streams take
~1x a spin's time on separate queues and ~2x on a shared one.  Streams: the caller's (null)
stream, then pool streams p0..p7 in torch.cuda.Stream() order."""
import time

import torch

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
null = torch.cuda.current_stream(dev)
pool = [torch.cuda.Stream(dev) for _ in range(8)]
names = ["null"] + [f"p{i}" for i in range(8)]
streams = [null] + pool
CYC = int(5e7)


def run(ss):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for s in ss:
        with torch.cuda.stream(s):
            torch.cuda._sleep(CYC)
    torch.cuda.synchronize()
    return time.perf_counter() - t


run([null])
one = min(run([null]) for _ in range(3))
print(f"one spin {one * 1e3:.2f} ms")
for i in range(len(streams)):
    row = []
    for j in range(len(streams)):
        row.append("  -" if i == j else f"{run([streams[i], streams[j]]) / one:4.1f}")
    print(f"{names[i]:>5}", " ".join(row))
for group in ([0, 1, 2, 3], [1, 2, 3, 4], [0, 1, 2], [1, 2, 3], [5, 6, 7, 8]):
    print("group", [names[k] for k in group], f"{run([streams[k] for k in group]) / one:.2f}")
