import torch, time
a = torch.empty(1648 * 1024 * 1024 // 2, dtype=torch.bfloat16, device="cuda").normal_()
b = torch.empty_like(a)
for name, fn, nbytes in [("copy", lambda: b.copy_(a), 2 * a.numel() * 2), ("read_sum", lambda: a.sum(), a.numel() * 2), ("fill", lambda: b.fill_(1.0), b.numel() * 2)]:
    for _ in range(3): fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10): fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    print(f"{name}: {nbytes / dt / 1e12:.2f} TB/s ({dt * 1e6:.0f} us)")
