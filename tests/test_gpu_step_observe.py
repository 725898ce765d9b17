"""oth_step_observe / oth_sample_step_observe: the observation OthelloBaseEnv.step
returns (othello.py:462), or any oth_observe layout, written by the launch that
stepped the boards.  Bit for bit equal to the oracle's step followed by the
oracle's observation (oracle_observe: get_observation / make_state,
othello.py:363-378, util.py:48-74) and to the two-call form (oth_step +
oth_observe, oth_sample_step + oth_observe).  Run on an MI355X (`-m gpu`)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

LAYOUTS = ("board", "board_legal", "make_state", "absolute", "legal")


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _dtypes(torch):
    return (torch.int8, torch.int32, torch.int64, torch.float32, torch.float64, torch.bfloat16)


def host(o):
    """An observation on the host as numpy (bfloat16, which numpy lacks, as
    float32: -1 / 0 / +1 are exact in both); bfloat16's bit patterns checked."""
    import torch
    if o.dtype == torch.bfloat16:
        bits = o.view(torch.int16).cpu().numpy()
        assert np.isin(bits, [0, 0x3F80, 0xBF80 - 0x10000]).all(), "bfloat16 -1 / 0 / +1 bit patterns"
        return o.float().cpu().numpy()
    return o.cpu().numpy()


def make_env(E, n, sd=True, auto=True, seed=9, init_rand=0):
    from gymothelloenv_amd import VecOthelloEnv
    return VecOthelloEnv(E, board_size=n, sudden_death_on_invalid_move=sd, auto_reset=auto, seed=seed,
                         initial_rand_steps=init_rand, device="cuda:0")


def oracle_obs(s, layout):
    """The oracle's observation of State s in `layout`: get_observation (1 and 2
    planes) and make_state from oracle_observe (othello_oracle.c); board_state
    (othello.py:257) and the possible_moves plane from the state's bits."""
    n, E, W = s.n, s.E, s.W
    if layout in ("board", "board_legal", "make_state"):
        obs, obs2, ms = oracle.observe(s)
        return {"board": obs, "board_legal": obs2, "make_state": ms}[layout]
    sq = np.arange(n * n)

    def bits(words):
        return ((words[:, sq // 64] >> (sq % 64).astype(np.uint64)) & np.uint64(1)).astype(np.int64)
    if layout == "absolute":
        return (bits(s.boards[:, W:]) - bits(s.boards[:, :W])).reshape(E, n, n)
    return bits(s.legal).reshape(E, n, n)


def legal_bool(legal, n):
    a = np.arange(n * n)
    return ((legal[:, a // 64] >> (a % 64).astype(np.uint64)) & np.uint64(1)).astype(bool)


def mixed_actions(rng, s, n):
    """Legal moves, with 10 % illegal / out-of-range ones (and every board
    without a legal move) taking the invalid path."""
    E = s.E
    lb = legal_bool(s.legal, n)
    pick = np.argmax(rng.rand(E, n * n) * lb, axis=1).astype(np.int32)
    wild = (rng.rand(E) < 0.1) | ~lb.any(axis=1)
    return np.where(wild, rng.randint(-2, n * n + 2, size=E), pick).astype(np.int32)


def state_np(env):
    b, m, lg = env.get_state()
    return b.cpu().numpy().view(np.uint64), m.cpu().numpy().view(np.uint16), lg.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("n,E", [(8, 65536), (8, 70001), (6, 20000), (4, 777), (8, 1), (10, 5000), (7, 3001),
                                 (10, 70001), (12, 1001), (16, 257), (9, 999)])
def test_step_observe_every_layout_and_dtype(torch_cuda, n, E):
    """step(observe=True) through oth_step_observe (one launch for one-word boards
    with N*N % 4 == 0: k_ply_step_obs; oth_step's kernel + k_observe otherwise)
    in both sudden-death modes with auto-reset: rewards, dones and the
    observation of every layout and dtype (one combination per ply, every
    combination in each mode) equal the oracle's step and observation."""
    torch = torch_cuda
    combos = [(lay, dt) for lay in LAYOUTS for dt in _dtypes(torch)]
    for sd in (True, False):
        flags = (oracle.F_SUDDEN_DEATH if sd else 0) | oracle.F_AUTO_RESET
        rng = np.random.RandomState(E + n + sd)
        env = make_env(E, n, sd=sd)
        s = oracle.reset(n, E)
        dbuf = torch.empty(E, dtype=torch.bool, device="cuda")  # dones as a bool tensor, written in place
        for p in range(len(combos)):
            layout, dt = combos[(p + 7 * sd) % len(combos)]
            acts = mixed_actions(rng, s, n)
            orw, od, _ = oracle.step(s, flags, acts, seed=9, ply=p)
            obs, rew, dn, _ = env.step(torch.from_numpy(acts).cuda(), dones=dbuf, obs_layout=layout, obs_dtype=dt)
            what = "%dx%d E=%d sd=%d ply %d %s %s" % (n, n, E, sd, p, layout, dt)
            np.testing.assert_array_equal(rew.cpu().numpy(), orw, err_msg=what)
            np.testing.assert_array_equal(dn.cpu().numpy(), od.astype(bool), err_msg=what)
            assert obs.dtype == dt
            h = host(obs)
            np.testing.assert_array_equal(h, oracle_obs(s, layout).astype(h.dtype), err_msg=what)
        b, m, lg = state_np(env)
        np.testing.assert_array_equal(b, s.boards)
        np.testing.assert_array_equal(m, s.meta)
        np.testing.assert_array_equal(lg, s.legal)
        env.close()


@pytest.mark.parametrize("n,E", [(8, 65536), (6, 4099), (8, 262147)])
def test_step_observe_equals_two_calls_and_default_layout(torch_cuda, n, E):
    """The fused call against oth_step + oth_observe on a twin handle: equal
    rewards, dones, state, W/D/L and observation; the default observation is
    get_observation()'s (board, or board_legal with possible_actions_in_obs);
    an output one element past the vector alignment takes the two-launch path
    with the same values; preallocated outputs are written in place.  From
    262,144 boards the fused launch takes one lane per board, 64 boards a wave."""
    torch = torch_cuda
    from gymothelloenv_amd import VecOthelloEnv
    for pa in (False, True):
        kw = dict(board_size=n, auto_reset=True, seed=4, possible_actions_in_obs=pa, device="cuda:0")
        fused, split = VecOthelloEnv(E, **kw), VecOthelloEnv(E, **kw)
        rng = np.random.RandomState(n + pa)
        s = oracle.reset(n, E)
        planes = 2 if pa else 1
        shape = (E, planes, n, n) if pa else (E, n, n)
        buf = torch.empty(E * planes * n * n + 1, dtype=torch.int64, device="cuda")
        off = buf[1:].view(shape)  # past the 4-element alignment: two launches
        rew = torch.empty(E, dtype=torch.int32, device="cuda")
        for p in range(12):
            acts = mixed_actions(rng, s, n)
            oracle.step(s, oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET, acts, seed=4, ply=p)
            a = torch.from_numpy(acts).cuda()
            if p % 2:
                o1, r1, d1, _ = fused.step(a, rewards=rew, obs=off)
                assert o1 is off and r1 is rew
            else:
                o1, r1, d1, _ = fused.step(a)
            _, r2, d2, _ = split.step(a, observe=False)
            o2 = split.get_observation()
            assert tuple(o1.shape) == shape and o1.dtype == torch.int64
            assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(d1, d2), "ply %d pa=%d" % (p, pa)
        for x, y in zip(fused.get_state(), split.get_state()):
            assert torch.equal(x, y)
        assert torch.equal(fused.counts(), split.counts())
        assert int(fused.counts().sum()) > 0 or E < 10
        fused.close()
        split.close()


def test_step_observe_large_launch_every_layout(torch_cuda):
    """From 262,144 boards the fused launch takes one lane per board and 64 boards
    a wave (k_ply_step_obs<8, 1, 64>): every layout and dtype equal to oth_step
    + oth_observe on a twin handle (compared on the device), 262,147 boards."""
    torch = torch_cuda
    from gymothelloenv_amd import VecOthelloEnv
    E, n = 262147, 8
    kw = dict(board_size=n, auto_reset=True, seed=6, device="cuda:0")
    fused, split = VecOthelloEnv(E, **kw), VecOthelloEnv(E, **kw)
    rng = np.random.RandomState(3)
    s = oracle.reset(n, E)
    combos = [(lay, dt) for lay in LAYOUTS for dt in _dtypes(torch)]
    for p, (lay, dt) in enumerate(combos):
        acts = mixed_actions(rng, s, n)
        oracle.step(s, oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET, acts, seed=6, ply=p)
        a = torch.from_numpy(acts).cuda()
        o1, r1, d1, _ = fused.step(a, obs_layout=lay, obs_dtype=dt)
        _, r2, d2, _ = split.step(a, observe=False)
        o2 = split.observe(lay, dt)
        assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(d1, d2), "ply %d %s %s" % (p, lay, dt)
    b, m, lg = state_np(fused)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)
    fused.close()
    split.close()


@pytest.mark.parametrize("n", [8, 6])
def test_step_observe_on_terminated_boards(torch_cuda, n):
    """Without auto-reset, boards that are already terminated stay as they were
    (the reference raises ValueError there; batched: a no-op reporting done)
    and the fused observation shows them unchanged (the kernel restores the
    registers its step changed)."""
    torch = torch_cuda
    E = 4096
    env = make_env(E, n, auto=False, seed=2)
    s = oracle.reset(n, E)
    rng = np.random.RandomState(n)
    flags = oracle.F_SUDDEN_DEATH
    for p in range(n * n):
        acts = mixed_actions(rng, s, n)
        orw, od, _ = oracle.step(s, flags, acts, seed=2, ply=p)
        lay = LAYOUTS[p % len(LAYOUTS)]
        obs, rew, dn, _ = env.step(torch.from_numpy(acts).cuda(), obs_layout=lay, obs_dtype=torch.int32)
        np.testing.assert_array_equal(rew.cpu().numpy(), orw)
        np.testing.assert_array_equal(dn.cpu().numpy(), od.astype(bool))
        np.testing.assert_array_equal(obs.cpu().numpy(), oracle_obs(s, lay).astype(np.int32), err_msg="ply %d" % p)
    _, m, _ = state_np(env)
    assert ((m >> 1) & 1).sum() > E // 2  # most boards ended and were stepped again while terminated


@pytest.mark.parametrize("n,E,lay,dt", [(8, 65536, "make_state", "float32"), (8, 4096, "make_state", "float32"),
                                        (8, 65536, "make_state", "int8"), (8, 65536, "make_state", "bfloat16"),
                                        (8, 16384, "make_state", "bfloat16"), (6, 20000, "make_state", "int8"),
                                        (8, 70001, "board", "int64"), (6, 20000, "make_state", "float64"),
                                        (10, 5000, "board_legal", "int8"), (7, 3001, "make_state", "float32"),
                                        (12, 999, "board", "int32")])
def test_sample_step_observe(torch_cuda, n, E, lay, dt):
    """sample_step(observe=layout): the masked sample, the step and the stepped
    boards' observation in one launch (lane pairs at 8x8 beyond 16,384 boards
    and 10x10, lane quads up to 16,384, one lane per board at 6x6 / 12x12; odd N
    two launches) equal sample_actions + step + observe on a twin handle, and
    the step and observation equal the oracle's."""
    torch = torch_cuda
    from gymothelloenv_amd import VecOthelloEnv
    dtype = getattr(torch, dt)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(n + E)
    kw = dict(board_size=n, auto_reset=True, seed=3, device=dev)
    fused, split = VecOthelloEnv(E, **kw), VecOthelloEnv(E, **kw)
    s = oracle.reset(n, E)
    for k in range(6):
        logits = torch.randn(E, n * n, device=dev, generator=g) * 3
        a1, lp1, en1, r1, d1, o1 = fused.sample_step(logits, observe=lay, obs_dtype=dtype)
        a2, lp2, en2 = split.sample_actions(logits)
        _, r2, d2, _ = split.step(a2, observe=False)
        o2 = split.observe(lay, dtype)
        what = "%dx%d E=%d ply %d" % (n, n, E, k)
        assert torch.equal(a1, a2) and torch.equal(lp1, lp2) and torch.equal(en1, en2), what + ": sampler"
        assert torch.equal(r1, r2) and torch.equal(d1, d2), what + ": step"
        assert o1.dtype == dtype and torch.equal(o1, o2), what + ": observation"
        orw, od, _ = oracle.step(s, oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET, a1.cpu().numpy(), seed=3, ply=k)
        np.testing.assert_array_equal(r1.cpu().numpy(), orw, err_msg=what)
        h = host(o1)
        np.testing.assert_array_equal(h, oracle_obs(s, lay).astype(h.dtype), err_msg=what)
    for x, y in zip(fused.get_state(), split.get_state()):
        assert torch.equal(x, y)
    assert torch.equal(fused.counts(), split.counts())  # the per-wave W/D/L slots
    fused.close()
    split.close()


def test_step_output_buffers_checked(torch_cuda):
    """Caller-given rewards / dones / obs of the wrong dtype, size, device or
    layout raise ValueError before any launch; good buffers are
    accepted and reused."""
    torch = torch_cuda
    E = 1000
    env = make_env(E, 8)
    a = torch.zeros(E, dtype=torch.int32, device="cuda")
    bad = [dict(rewards=torch.zeros(E, dtype=torch.int64, device="cuda")),
           dict(rewards=torch.zeros(E - 1, dtype=torch.int32, device="cuda")),
           dict(rewards=torch.zeros(2 * E, dtype=torch.int32, device="cuda")[::2]),
           dict(rewards=torch.zeros(E, dtype=torch.int32)),
           dict(dones=torch.zeros(E, dtype=torch.int32, device="cuda")),
           dict(dones=torch.zeros(E + 1, dtype=torch.uint8, device="cuda")),
           dict(obs=torch.zeros(E, 8, 8, dtype=torch.int16, device="cuda")),
           dict(obs=torch.zeros(E, 8, 7, dtype=torch.int64, device="cuda")),
           dict(obs=torch.zeros(E, 8, 8, dtype=torch.int64, device="cuda"), obs_layout="make_state")]
    b0 = state_np(env)
    for kw in bad:
        with pytest.raises(ValueError):
            env.step(a, **kw)
    for x, y in zip(state_np(env), b0):
        np.testing.assert_array_equal(x, y)  # nothing was launched
    r = torch.empty(E, dtype=torch.int32, device="cuda")
    d = torch.empty(E, dtype=torch.uint8, device="cuda")
    o = torch.empty(E, 4, 8, 8, dtype=torch.float32, device="cuda")
    for _ in range(3):
        obs, rr, dd, _ = env.step(a, rewards=r, dones=d, obs=o, obs_layout="make_state")
        assert obs is o and rr is r
    env.close()


@pytest.mark.parametrize("n,opp,E", [(8, "random", 65536), (8, "greedy", 4099), (6, "random", 3000),
                                     (10, "greedy", 2000), (8, "maximin2", 1000)])
def test_step_vs_observe_equals_two_calls(torch_cuda, n, opp, E):
    """OthelloEnv.step on the device with its returned observation (othello.py:200)
    from the same launch (k_step_vs1 + the observation tail; the generic k_step_vs
    and a k_observe launch for two-word boards and MaxiMin opponents): every
    layout equal to oth_step_vs + oth_observe on a twin handle, mixed protagonist
    colours, random openings, auto-reset."""
    torch = torch_cuda
    from gymothelloenv_amd import VecOthelloEnv
    kw = dict(board_size=n, auto_reset=True, seed=12, initial_rand_steps=4, device="cuda:0")
    fused, split = VecOthelloEnv(E, **kw), VecOthelloEnv(E, **kw)
    prot = torch.from_numpy(np.where(np.arange(E) % 3 == 0, -1, 1).astype(np.int8))
    o1 = fused.reset_vs(opp, protagonist=prot)
    o2 = split.reset_vs(opp, protagonist=prot)
    assert torch.equal(o1, o2)
    for c in range(12):
        acts = fused.policy_actions("greedy")
        lay, dt = LAYOUTS[c % len(LAYOUTS)], _dtypes(torch)[c % 6]
        o1, r1, d1, p1 = fused.step_vs(acts, opp, obs_layout=lay, obs_dtype=dt)
        _, r2, d2, p2 = split.step_vs(acts, opp, observe=False)
        o2 = split.observe(lay, dt)
        what = "%s %dx%d call %d %s %s" % (opp, n, n, c, lay, dt)
        assert torch.equal(r1, r2) and torch.equal(d1, d2) and torch.equal(p1, p2), what
        assert o1.dtype == dt and torch.equal(o1, o2), what
    for x, y in zip(fused.get_state(), split.get_state()):
        assert torch.equal(x, y)
    assert torch.equal(fused.counts_vs(), split.counts_vs())
