# Variant bisection for the greedy rollout (N=8, random openings): every named build in
# gymothelloenv_amd/variants/ replays 140 greedy plies against the oracle (one launch and
# one launch per ply) and checks random play split over launches.  GPU box only:
#   python tools/ab_variants.py --build a= b=-DOTH_GREEDY_WORD64=0   (here)
#   python tools/bisect_greedy.py a b                               (gpurun)
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from gymothelloenv_amd import _lib as L
from gymothelloenv_amd import VecOthelloEnv
from oracle import oracle

VDIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gymothelloenv_amd", "variants")
n, E, seed, ir, plies = 8, 2048, 11, 10, 140
flags = oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET
s = oracle.reset_openings(n, E, seed, 0, 0, ir)
oa, orw, od, owdl = oracle.rollout(s, flags, 1, plies, seed=seed, initial_rand_steps=ir)
for nm in sys.argv[1:]:
    lib = L.load_path(os.path.join(VDIR, "liboth_%s.so" % nm))
    for pol in ("greedy", "random"):
        env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=seed, initial_rand_steps=ir, device="cuda:0", lib=lib)
        env.reset()
        if pol == "random":
            a1, _, _ = env.step_policy("random", n_plies=60)
            env2 = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=seed, initial_rand_steps=ir, device="cuda:0", lib=lib)
            env2.reset()
            a2 = torch.cat([env2.step_policy("random", n_plies=1)[0] for _ in range(60)])
            print(nm, pol, "multi==single", bool(torch.equal(a1, a2)), flush=True)
            continue
        a, r, d = env.step_policy(pol, n_plies=plies)
        a = a.cpu().numpy()
        bad = np.argwhere(a != oa)
        print(nm, pol, "mismatches", len(bad), "first", bad[:3].tolist() if len(bad) else None, flush=True)
        # greedy again, one ply per launch, from the same start
        env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=seed, initial_rand_steps=ir, device="cuda:0", lib=lib)
        env.reset()
        a2 = np.concatenate([env.step_policy(pol, n_plies=1)[0].cpu().numpy() for _ in range(plies)])
        bad = np.argwhere(a2 != oa)
        print(nm, pol, "1-ply launches mismatches", len(bad), "first", bad[:3].tolist() if len(bad) else None, flush=True)
print("done")
