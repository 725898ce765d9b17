# The dword-pair (U2) greedy planes miscompile: find the first
# wrong greedy move of a variant build, then replay that one position alone
# (E = 1) through k_play (1 ply) and k_policy_actions, next to the oracle.
#   python tools/ab_variants.py --build g0=-DOTH_GREEDY_WORD64=0 ...   (here)
#   python tools/bisect_u2.py g0 [g0o1 ...]                           (gpurun)
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gymothelloenv_amd import _lib as L
from gymothelloenv_amd import VecOthelloEnv
from oracle import oracle

VDIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gymothelloenv_amd", "variants")
n, E, seed, ir, plies = 8, 2048, 11, 10, 140
flags = oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET
s = oracle.reset_openings(n, E, seed, 0, 0, ir)
oa, _, _, _ = oracle.rollout(s.copy(), flags, 1, plies, seed=seed, initial_rand_steps=ir)
for nm in sys.argv[1:]:
    lib = L.load_path(os.path.join(VDIR, "liboth_%s.so" % nm))
    env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=seed, initial_rand_steps=ir, device="cuda:0", lib=lib)
    env.reset()
    a = env.step_policy("greedy", n_plies=plies)[0].cpu().numpy()
    bad = np.argwhere(a != oa)
    print(nm, "mismatches", len(bad), "first", bad[:2].tolist() if len(bad) else None, flush=True)
    if not len(bad):
        continue
    p, e = (int(v) for v in bad[0])
    pre = s.copy()
    oracle.rollout(pre, flags, 1, p, seed=seed, initial_rand_steps=ir)  # state before ply p
    b, m, lg = pre.boards[e:e + 1].copy(), pre.meta[e:e + 1].copy(), pre.legal[e:e + 1].copy()
    one = oracle.State(n, 1)
    one.boards[:], one.meta[:], one.legal[:] = b, m, lg
    ref = oracle.greedy(one)[0]
    tw = int(m[0]) & 1
    mover, opp = (int(b[0, 1]), int(b[0, 0])) if tw else (int(b[0, 0]), int(b[0, 1]))
    print(" position: black %#018x white %#018x meta %#06x legal %#018x mover %s" %
          (int(b[0, 0]), int(b[0, 1]), int(m[0]), int(lg[0, 0]), "white" if tw else "black"))
    print(" oracle greedy", ref, "k_play(E=%d) gave" % E, int(a[p, e]), "rand_left", int(m[0]) >> 8)
    for label, E1 in (("E=1", 1), ("E=64", 64)):
        env1 = VecOthelloEnv(E1, board_size=n, auto_reset=True, seed=seed, initial_rand_steps=0, device="cuda:0",
                             lib=lib)
        t = lambda x: torch.from_numpy(np.repeat(x, E1, axis=0).view(np.int64) if x.dtype == np.uint64
                                       else np.repeat(x, E1, axis=0).view(np.int16)).cuda()
        env1.set_state(t(b), t(m & 0x00ff), t(lg))
        pa = env1.policy_actions("greedy").cpu().numpy()
        env1.set_state(t(b), t(m & 0x00ff), t(lg))
        ka = env1.step_policy("greedy", n_plies=1)[0].cpu().numpy()[0]
        print(" ", label, "k_policy_actions", sorted(set(pa.tolist())), "k_play 1 ply", sorted(set(ka.tolist())), flush=True)
print("done")
