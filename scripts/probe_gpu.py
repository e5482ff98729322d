"""One-off GPU probe: device info + a quick plain-PyTorch ResNet-50 (CIFAR stem) step timing."""
import time, torch, torch.nn as nn, torch.nn.functional as F
print("torch", torch.__version__, "hip", torch.version.hip, "avail", torch.cuda.is_available())
p = torch.cuda.get_device_properties(0)
print(p)
dev = "cuda"
# GEMM speed check
for (m, k, n) in [(8192, 8192, 8192), (1048576, 64, 256), (1048576, 256, 64), (65536, 1024, 256)]:
    a = torch.randn(m, k, device=dev, dtype=torch.bfloat16); b = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
    for _ in range(3): c = a @ b
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(10): c = a @ b
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 10
    print(f"mm {m}x{k}x{n}: {dt*1e3:.3f} ms  {2*m*k*n/dt/1e12:.1f} TF  {(m*k+k*n+m*n)*2/dt/1e12:.2f} TB/s")
# conv speed check, channels_last bf16
for (n, c, h, k, r) in [(1024, 64, 32, 64, 3), (1024, 128, 16, 128, 3), (1024, 256, 8, 256, 3), (1024, 512, 4, 512, 3)]:
    x = torch.randn(n, c, h, h, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    w = torch.randn(k, c, r, r, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    for _ in range(3): y = F.conv2d(x, w, padding=1)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(10): y = F.conv2d(x, w, padding=1)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 10
    fl = 2 * n * h * h * c * k * r * r
    print(f"conv3x3 n{n} c{c} h{h} k{k}: {dt*1e3:.3f} ms {fl/dt/1e12:.1f} TF")
