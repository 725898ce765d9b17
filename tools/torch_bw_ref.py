import torch, json
for E in (1048576, 4194304):
    x = torch.randn(E, 64, device="cuda")
    for name, fn in (("amax", lambda: torch.amax(x, dim=1)), ("sum", lambda: x.sum(1)), ("copy", lambda: x.clone())):
        for _ in range(3): fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50): fn()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        b = E * 256 * (2 if name == "copy" else 1)
        print(json.dumps({"op": name, "E": E, "us": us, "GBs": b / us / 1e3}))
