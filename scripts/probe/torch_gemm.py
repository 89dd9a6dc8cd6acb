"""Times torch.nn.functional.linear (hipBLASLt) on the ViT-L/14 bs=256 GEMM shapes, for
rocprofv3 kernel-name / duration comparison with gemm.hip (diagnostic only)."""
import torch
M, W = 256 * 257, 1024
g = torch.Generator(device="cuda").manual_seed(0)
A = (torch.randn(M, 4 * W, device="cuda", generator=g) * 0.5).half()
Wt = (torch.randn(4 * W, 4 * W, device="cuda", generator=g) * 0.02).half()
b = torch.randn(4 * W, device="cuda", generator=g).half()
for N, K in ((3 * W, W), (W, W), (4 * W, W), (W, 4 * W)):
    a_, w_, b_ = A[:, :K].contiguous(), Wt[:N, :K].contiguous(), b[:N].contiguous()
    for _ in range(10):
        torch.nn.functional.linear(a_, w_)
        torch.nn.functional.linear(a_, w_, b_)
    torch.cuda.synchronize()
