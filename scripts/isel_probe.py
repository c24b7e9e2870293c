import time, torch
d = torch.device("cuda")
x = torch.randn(3000, 6, device=d)
for dt in (torch.int32, torch.int64):
    idx = torch.randint(0, 3000, (40,), device=d, dtype=dt)
    for _ in range(10): x.index_select(0, idx)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(200): x.index_select(0, idx)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(dt, f"host {(t1 - t) / 200 * 1e6:.1f} us/call")
    idx2 = idx[5:30]
    t = time.perf_counter()
    for _ in range(200): x.index_select(0, idx2)
    print(dt, "slice idx", f"{(time.perf_counter() - t) / 200 * 1e6:.1f} us/call")
