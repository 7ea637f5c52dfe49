import sys, torch, time
sys.path.insert(0, "/root/repo/multimodal-baselines_amd")
import mmb_lib as L
dev = torch.device("cuda", 0)
for B in (8, 64, 512):
    x = torch.randn(B, 300, device=dev)
    w1 = torch.randn(100, 300, device=dev); b1 = torch.randn(100, device=dev)
    w2 = torch.randn(1, 100, device=dev); b2 = torch.randn(1, device=dev)
    y = torch.empty(B, 1, device=dev); hid = torch.empty(B, 100, device=dev)
    f = lambda: L.call("mmb_mlp_forward_train", L.ptr(x), B, 300, 100, 1, L.ptr(w1), L.ptr(b1), L.ptr(w2), L.ptr(b2), L.ptr(y), L.ptr(hid), L.stream_ptr())
    for _ in range(5): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200): f()
    e1.record(); torch.cuda.synchronize()
    ref = torch.relu(x @ w1.t() + b1) @ w2.t() + b2
    print(B, "us per call", e0.elapsed_time(e1) / 200 * 1e3, "max err", (ref - y).abs().max().item())
