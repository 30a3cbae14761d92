"""Reference point only: torch.matmul (hipBLASLt) bf16 timings on the step's GEMM shapes."""
import json
import torch

BT = 32 * 251
SHAPES = [("in-proj L1-3", BT, 2400, 600), ("Linear", BT, 6450, 600), ("dW_lin", 6450, 600, BT),
          ("dH", BT, 600, 6450), ("dW_ih", 2400, 600, BT), ("dX", BT, 600, 2400), ("dW_hh", 1200, 300, BT)]
dev = torch.device("cuda")
for name, M, N, K in SHAPES:
    for dt in (torch.bfloat16, torch.float32):
        A = torch.randn(M, K, device=dev, dtype=dt)
        B = torch.randn(K, N, device=dev, dtype=dt)
        for _ in range(3):
            C = A @ B
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            C = A @ B
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 20
        print(json.dumps({"gemm": name, "dtype": str(dt), "us": round(ms * 1e3, 1),
                          "TFLOP/s": round(2 * M * N * K / ms / 1e9, 1)}), flush=True)
