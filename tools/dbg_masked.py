import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from gymothelloenv_amd import VecOthelloEnv, masked_sample
from gymothelloenv_amd import _lib as L
lib = L.load_path(sys.argv[1]) if len(sys.argv) > 1 else None
print("lib", sys.argv[1:])
E = 2048
env = VecOthelloEnv(E, board_size=8, seed=11, device="cuda:0", lib=lib)
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
for ply in range(70):
    logits = torch.randn(E, 64, device="cuda", generator=g) * 2
    legal = env.legal_mask()
    a, lp, ent = env.sample_actions(logits)
    lpn = lp.cpu().numpy()
    bad = np.flatnonzero(~(lpn <= 0))
    if len(bad): print("ply", ply, "bad", len(bad), lpn[bad][:5])
    L = legal.cpu().numpy().view(np.uint64)[:, 0]
    for i in bad[:1]:
        row = logits[i].cpu().numpy()
        lg = [b for b in range(64) if (int(L[i]) >> b) & 1]
        x = row[lg]
        m = x.max()
        print(" row", i, "a", int(a[i]), "legal", lg, "x", x, "lp", lpn[i], "ref", row[int(a[i])] - m - np.log(np.exp(x - m).sum()), "ent", float(ent[i]))
    env.step(a, observe=False)
for mode in ("mode", "sample"):
    acts, lp2, ent2 = masked_sample(logits, legal, 8, mode=mode, lib=lib)
    print(mode, "bad", int((~(lp2 <= 0)).sum()))
