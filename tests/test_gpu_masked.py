"""Masked categorical over legal squares (csrc/masked.hip)
against a float64 numpy restatement of the learners' per-sample loops
(model.py:60-99 act, :156-178 evaluate_actions; ppo.py:228-298 get_action)
and torch's own Categorical (the reference's FixedCategorical base class).

Tolerances (fp32 kernel vs fp64 restatement): log-probs and entropies
atol 2e-5 + rtol 1e-5; a sampled square may differ from the fp64 choice only
when u * total lies within 1e-5 * total of a cumulative-mass boundary."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [4, 5, 6, 7, 8, 10, 16]
ATOL, RTOL, CDF_TOL = 2e-5, 1e-5, 1e-5


@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def pack(legal_bool):
    """(n, N*N) bool -> (n, W) int64 bit masks (bit a of word a // 64 = square a)."""
    n, nn = legal_bool.shape
    w = (nn + 63) // 64
    out = np.zeros((n, w), dtype=np.uint64)
    for a in range(nn):
        out[:, a // 64] |= legal_bool[:, a].astype(np.uint64) << np.uint64(a % 64)
    return out.view(np.int64)


def make_case(rng, n, nn):
    logits = (rng.standard_normal((n, nn)) * 3).astype(np.float32)
    legal = rng.random((n, nn)) < rng.uniform(0.05, 0.5, size=(n, 1))
    legal[: n // 16] = False                    # no legal move
    one = slice(n // 16, n // 8)                # exactly one legal move
    legal[one] = False
    legal[one, rng.integers(0, nn, size=n // 8 - n // 16)] = True
    ties = slice(n // 8, n // 8 + n // 32)      # equal logits: mode takes the lowest square
    logits[ties] = 1.25
    return logits, legal


def ref_masked(logits, legal, u):
    """fp64 restatement: masked softmax, first-max mode, np.random.choice's
    searchsorted(cdf, u * total, 'right'), log-prob and entropy."""
    x = logits.astype(np.float64)
    anyl = legal.any(1)
    m = np.where(legal, x, -np.inf).max(1)
    m = np.where(anyl, m, 0.0)
    p = np.where(legal, np.exp(x - m[:, None]), 0.0)
    S = p.sum(1)
    lse = m + np.log(np.where(anyl, S, 1.0))
    mode = np.argmax(np.where(legal, x, -np.inf), axis=1)
    cdf = np.cumsum(p, 1)
    target = u * S
    hit = (cdf > target[:, None]) & legal
    samp = np.where(hit.any(1), np.argmax(hit, 1), legal.shape[1] - 1 - np.argmax(legal[:, ::-1], 1))
    mode = np.where(anyl, mode, 0)
    samp = np.where(anyl, samp, 0)
    ent = np.where(anyl, -(np.where(legal, p / np.where(anyl, S, 1.0)[:, None], 0.0) *
                           np.where(legal, x - lse[:, None], 0.0)).sum(1), 0.0)
    return dict(mode=mode, samp=samp, lse=lse, ent=ent, cdf=cdf, p=p, S=S, target=target, x=x, anyl=anyl)


def lp_of(ref, legal, a):
    rows = np.arange(len(a))
    ok = ref["anyl"] & (a >= 0) & (a < legal.shape[1])
    ok[ok] &= legal[rows[ok], a[ok]]
    return np.where(ok, ref["x"][rows, np.clip(a, 0, legal.shape[1] - 1)] - ref["lse"], 0.0)


@pytest.mark.parametrize("n_board", SIZES)
def test_masked_matches_fp64_restatement(torch_gpu, n_board):
    torch = torch_gpu
    from gymothelloenv_amd import masked_log_prob, masked_sample
    rng = np.random.default_rng(n_board)
    n, nn = 4096, n_board * n_board
    logits, legal = make_case(rng, n, nn)
    u = rng.random(n).astype(np.float32)
    ref = ref_masked(logits, legal, u.astype(np.float64))
    dl = torch.from_numpy(logits).cuda()
    dg = torch.from_numpy(pack(legal)).cuda()
    # mode
    a, lp, ent = masked_sample(dl, dg, n_board, mode="mode")
    a = a.cpu().numpy()
    np.testing.assert_array_equal(a, ref["mode"])
    np.testing.assert_allclose(lp.cpu().numpy(), lp_of(ref, legal, a), atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(ent.cpu().numpy(), ref["ent"], atol=ATOL, rtol=RTOL)
    # sample with the caller's uniforms
    a, lp, ent = masked_sample(dl, dg, n_board, uniforms=torch.from_numpy(u).cuda())
    a = a.cpu().numpy()
    rows = np.arange(n)
    bad = np.flatnonzero(a != ref["samp"])
    assert len(bad) <= n // 200, len(bad)
    for i in bad:  # only boundary cases, and always a legal square whose mass interval holds u * total
        g = a[i]
        assert legal[i, g]
        hi, lo = ref["cdf"][i, g], ref["cdf"][i, g] - ref["p"][i, g]
        tol = CDF_TOL * ref["S"][i]
        assert lo - tol <= ref["target"][i] <= hi + tol, (i, g, ref["samp"][i])
    np.testing.assert_allclose(lp.cpu().numpy(), lp_of(ref, legal, a), atol=ATOL, rtol=RTOL)
    assert (a[~ref["anyl"]] == 0).all() and (lp.cpu().numpy()[~ref["anyl"]] == 0).all()
    assert legal[rows[ref["anyl"]], a[ref["anyl"]]].all()
    # evaluate_actions: arbitrary actions incl. illegal / out of range -> 0
    acts = rng.integers(-2, nn + 2, size=n).astype(np.int32)
    acts[: n // 2] = ref["samp"][: n // 2]
    lp2, ent2 = masked_log_prob(dl, dg, torch.from_numpy(acts).cuda(), n_board)
    np.testing.assert_allclose(lp2.cpu().numpy(), lp_of(ref, legal, acts), atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(ent2.cpu().numpy(), ref["ent"], atol=ATOL, rtol=RTOL)


def test_log_prob_matches_torch_categorical(torch_gpu):
    """FixedCategorical (the reference's distribution class) is torch's
    Categorical: compare its fp32 log_prob / entropy row by row."""
    torch = torch_gpu
    from gymothelloenv_amd import masked_sample
    rng = np.random.default_rng(7)
    logits, legal = make_case(rng, 512, 64)
    a, lp, ent = masked_sample(torch.from_numpy(logits).cuda(), torch.from_numpy(pack(legal)).cuda(), 8)
    a, lp, ent = a.cpu().numpy(), lp.cpu().numpy(), ent.cpu().numpy()
    for i in range(512):
        idx = np.flatnonzero(legal[i])
        if len(idx) == 0:
            assert a[i] == 0 and lp[i] == 0 and ent[i] == 0
            continue
        d = torch.distributions.Categorical(logits=torch.from_numpy(logits[i, idx]))
        k = int(np.flatnonzero(idx == a[i])[0])
        assert abs(float(d.log_prob(torch.tensor(k))) - lp[i]) <= ATOL + RTOL * abs(lp[i])
        assert abs(float(d.entropy()) - ent[i]) <= ATOL + RTOL * abs(ent[i])


def test_philox_sampling_distribution(torch_gpu):
    """Philox-keyed sampling of one distribution over 262,144 boards follows
    the masked softmax; repeat calls with the same key agree, a new counter
    draws afresh."""
    torch = torch_gpu
    from gymothelloenv_amd import masked_sample
    n = 262144
    row = np.linspace(-2.0, 2.0, 64).astype(np.float32)
    legal = np.zeros(64, bool)
    legal[[0, 3, 9, 20, 27, 36, 44, 50, 61, 63]] = True
    dl = torch.from_numpy(np.tile(row, (n, 1))).cuda()
    dg = torch.from_numpy(pack(np.tile(legal, (n, 1)))).cuda()
    a1, _, _ = masked_sample(dl, dg, 8, seed=5, counter=1)
    a2, _, _ = masked_sample(dl, dg, 8, seed=5, counter=1)
    a3, _, _ = masked_sample(dl, dg, 8, seed=5, counter=2)
    assert torch.equal(a1, a2) and not torch.equal(a1, a3)
    a1 = a1.cpu().numpy()
    assert legal[a1].all()
    p = np.exp(row[legal] - row[legal].max())
    p /= p.sum()
    freq = np.bincount(a1, minlength=64)[legal] / n
    assert np.abs(freq - p).max() < 5 * np.sqrt(p.max() / n)


def test_strided_and_unaligned_rows(torch_gpu):
    """Row stride > N*N (ld) and rows not 16-byte aligned (scalar-load path)."""
    torch = torch_gpu
    from gymothelloenv_amd import masked_sample
    rng = np.random.default_rng(3)
    logits, legal = make_case(rng, 1024, 64)
    u = torch.from_numpy(rng.random(1024).astype(np.float32)).cuda()
    dg = torch.from_numpy(pack(legal)).cuda()
    base = masked_sample(torch.from_numpy(logits).cuda(), dg, 8, uniforms=u)
    wide = torch.zeros(1024, 81, dtype=torch.float32, device="cuda")  # ld 81, rows start at column 1
    wide[:, 1:65] = torch.from_numpy(logits).cuda()
    pad = torch.zeros(1024, 80, dtype=torch.float32, device="cuda")   # ld 80, 16-byte aligned rows
    pad[:, :64] = torch.from_numpy(logits).cuda()
    for view in (wide[:, 1:65], pad[:, :64]):
        got = masked_sample(view, dg, 8, uniforms=u)
        assert torch.equal(got[0], base[0])
        torch.testing.assert_close(got[1], base[1], atol=1e-6, rtol=0)


def test_env_rollout_with_sampled_actions(torch_gpu):
    """VecOthelloEnv.sample_actions feeds step() directly: every sampled move is
    legal, so no game ends by sudden death, and the boards still replay
    bit-exactly through the CPU oracle."""
    torch = torch_gpu
    from gymothelloenv_amd import VecOthelloEnv
    from oracle import oracle
    E = 2048
    env = VecOthelloEnv(E, board_size=8, seed=11, device="cuda:0")
    twin = VecOthelloEnv(E, board_size=8, seed=11, device="cuda:0")
    env.reset()
    twin.reset()
    s = oracle.reset(8, E)
    g = torch.Generator(device="cuda").manual_seed(0)
    for ply in range(70):
        logits = torch.randn(E, 64, device="cuda", generator=g) * 2
        legal = env.legal_mask().cpu().numpy().view(np.uint64)[:, 0]
        a, lp, ent = env.sample_actions(logits)
        assert torch.equal(a, twin.sample_actions(logits)[0])  # same key -> same draws
        an = a.cpu().numpy()
        live = (s.meta & 2) == 0
        has = legal != 0
        assert all((int(legal[i]) >> int(an[i])) & 1 for i in np.flatnonzero(live & has))
        assert (lp.cpu().numpy()[live & has] <= 0).all()
        act = np.where(live, an, 0).astype(np.int32)
        _, r, d, _ = env.step(torch.from_numpy(act).cuda(), observe=False)
        twin.step(torch.from_numpy(act).cuda(), observe=False)
        rr, dd, _ = oracle.step(s, oracle.F_SUDDEN_DEATH, act)
        np.testing.assert_array_equal(r.cpu().numpy(), rr)
        b, m, lg = env.get_state()
        np.testing.assert_array_equal(b.cpu().numpy().view(np.uint64), s.boards)
        np.testing.assert_array_equal(lg.cpu().numpy().view(np.uint64), s.legal)
    assert (s.meta & 2).all()  # every game finished within 70 plies, none by an illegal move


@pytest.mark.parametrize("n_board", [6, 8])
def test_masked_matches_reference_policy_heads(torch_gpu, golden_dir, n_board):
    """k_masked against the reference's own policy heads on fixed logits
    (tests/golden/masked.npz, made by gen_golden.py from model.py / ppo.py):
    Policy.act's mode and log-probs (model.py:60-99), the log-probs of
    Policy.act's torch samples, Policy.evaluate_actions' log-probs and
    unmasked entropy (:156-178), PPO.get_action's renormalised probabilities
    and its np.random.choice draw for the recorded uniform (ppo.py:228-262).
    fp32 kernel vs the reference's fp32 torch / float64 numpy: atol 2e-5 +
    rtol 1e-5; a sampled square may differ only where u lies within 1e-5 of a
    cumulative-probability boundary (u is rounded to fp32 for the kernel)."""
    import os
    torch = torch_gpu
    from gymothelloenv_amd import masked_log_prob, masked_sample
    d = np.load(os.path.join(golden_dir, "masked.npz"))
    k = "N%d_" % n_board
    logits, nl = d[k + "logits"], d[k + "nlegal"]
    R, nn = logits.shape
    dl = torch.from_numpy(logits).cuda()
    dg = torch.from_numpy(d[k + "legal"].view(np.int64)).cuda()
    # Policy.act(deterministic=True)
    a, lp, _ = masked_sample(dl, dg, n_board, mode="mode")
    np.testing.assert_array_equal(a.cpu().numpy(), d[k + "mode_action"])
    np.testing.assert_allclose(lp.cpu().numpy(), d[k + "mode_logp"], atol=ATOL, rtol=RTOL)
    # Policy.act(deterministic=False): log-prob of the reference's own samples
    lp, _ = masked_log_prob(dl, dg, torch.from_numpy(d[k + "sample_action"]).cuda(), n_board, entropy=False)
    np.testing.assert_allclose(lp.cpu().numpy(), d[k + "sample_logp"], atol=ATOL, rtol=RTOL)
    # Policy.evaluate_actions: log-probs (0 off the choices) and dist.entropy() of the unmasked head
    lp, ent = masked_log_prob(dl, dg, torch.from_numpy(d[k + "eval_action"]).cuda(), n_board, full_entropy=True)
    np.testing.assert_allclose(lp.cpu().numpy(), d[k + "eval_logp"], atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(ent.cpu().numpy(), d[k + "full_entropy"], atol=ATOL, rtol=RTOL)
    # PPO.get_action: probabilities renormalised over possible_moves
    words = d[k + "legal"]
    probs = np.zeros((R, nn))
    for sq in range(nn):
        lp_sq, _ = masked_log_prob(dl, dg, torch.full((R,), sq, dtype=torch.int32, device="cuda"), n_board,
                                   entropy=False)
        is_legal = ((words[:, sq // 64] >> np.uint64(sq % 64)) & np.uint64(1)).astype(bool)
        probs[:, sq] = np.where(is_legal, np.exp(lp_sq.cpu().numpy().astype(np.float64)), 0.0)
    live = nl > 0
    np.testing.assert_allclose(probs[live], d[k + "ppo_probs"][live], atol=ATOL, rtol=RTOL)
    # ... and np.random.choice's draw for the recorded uniform
    u = d[k + "ppo_u"]
    a, _, _ = masked_sample(dl, dg, n_board, uniforms=torch.from_numpy(u.astype(np.float32)).cuda(),
                            log_probs=False, entropy=False)
    a = a.cpu().numpy()
    ref = d[k + "ppo_action"]
    bad = np.flatnonzero(live & (a != ref))
    assert len(bad) <= R // 100, len(bad)
    for i in bad:
        cdf = np.cumsum(d[k + "ppo_probs"][i])
        assert np.min(np.abs(cdf - u[i])) < CDF_TOL, (i, a[i], ref[i])


@pytest.mark.parametrize("n_board,E", [(8, 65536), (6, 3001), (7, 2049), (5, 1500), (4, 999), (10, 4096),
                                       (9, 777), (11, 3001), (9, 40000), (16, 1000)])
def test_sample_step_equals_sample_then_step(torch_gpu, n_board, E):
    """oth_sample_step (one launch: k_masked's sampler + OthelloBaseEnv.step)
    is bit-identical to sample_actions followed by step: actions, log-probs,
    entropies, rewards, dones, the boards and the W/D/L tally, over several
    plies with Philox draws, caller uniforms, the mode and the unmasked
    entropy, ragged E included."""
    torch = torch_gpu
    from gymothelloenv_amd import VecOthelloEnv
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(n_board)
    kw = dict(board_size=n_board, auto_reset=True, initial_rand_steps=4, seed=3, device=dev)
    fused, split = VecOthelloEnv(E, **kw), VecOthelloEnv(E, **kw)
    fused.reset()
    split.reset()
    for k in range(12):
        logits = torch.randn(E, n_board * n_board, device=dev, generator=g) * 3
        uni = torch.rand(E, device=dev, generator=g) if k % 3 == 1 else None
        det, full = k % 4 == 2, k % 5 == 3
        a1, lp1, en1, r1, d1 = fused.sample_step(logits, deterministic=det, uniforms=uni, full_entropy=full)
        if full:
            a2, _, _ = split.sample_actions(logits, deterministic=det, uniforms=uni)
            from gymothelloenv_amd import masked_log_prob
            lp2, en2 = masked_log_prob(logits, split.legal_mask(), a2, n_board, full_entropy=True)
        else:
            a2, lp2, en2 = split.sample_actions(logits, deterministic=det, uniforms=uni)
        _, r2, d2, _ = split.step(a2, observe=False)
        assert torch.equal(a1, a2), k
        assert torch.equal(lp1, lp2) and torch.equal(en1, en2), k  # bit-identical floats
        assert torch.equal(r1, r2) and torch.equal(d1, d2), k
        for x, y in zip(fused.get_state(), split.get_state()):
            assert torch.equal(x, y), k
    assert torch.equal(fused.counts(), split.counts())
    assert fused.ply_counter == split.ply_counter and fused.sample_counter == split.sample_counter


def test_sample_step_graph_region_replays(torch_gpu):
    """The fused ply captured in a HIP graph inside graph_region: replay r
    equals the same fused plies run eagerly at the region's counters."""
    torch = torch_gpu
    from gymothelloenv_amd import VecOthelloEnv
    E, n, K = 4096, 8, 6
    dev = torch.device("cuda", 0)
    logits = torch.randn(E, n * n, device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    kw = dict(board_size=n, auto_reset=True, initial_rand_steps=2, seed=8, device=dev)
    eager, graphed = VecOthelloEnv(E, **kw), VecOthelloEnv(E, **kw)
    eager.reset()
    graphed.reset()
    out_g = torch.empty(K, E, dtype=torch.int32, device=dev)
    out_e = torch.empty_like(out_g)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph), graphed.graph_region() as slot:
        for k in range(K):
            out_g[k].copy_(graphed.sample_step(logits, log_probs=False, entropy=False)[0])
    torch.cuda.synchronize()
    for r in range(3):
        eager.ply_counter = eager.sample_counter = graphed.graph_counter_base(slot) + r * K
        for k in range(K):
            out_e[k].copy_(eager.sample_step(logits, log_probs=False, entropy=False)[0])
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out_g, out_e)
        for x, y in zip(graphed.get_state(), eager.get_state()):
            assert torch.equal(x, y)


def test_sample_step_writes_given_outputs(torch_gpu):
    """Outputs handed to sample_step are written in place and equal fresh ones;
    a wrong dtype / size is refused before any launch."""
    torch = torch_gpu
    from gymothelloenv_amd import VecOthelloEnv
    E, n = 1000, 8
    dev = torch.device("cuda", 0)
    logits = torch.randn(E, n * n, device=dev, generator=torch.Generator(device=dev).manual_seed(2))
    kw = dict(board_size=n, auto_reset=True, seed=4, device=dev)
    a, b = VecOthelloEnv(E, **kw), VecOthelloEnv(E, **kw)
    a.reset()
    b.reset()
    acts = torch.full((E,), -7, dtype=torch.int32, device=dev)
    lp = torch.empty(E, device=dev)
    ent = torch.empty(E, device=dev)
    rew = torch.empty(E, dtype=torch.int32, device=dev)
    don = torch.empty(E, dtype=torch.uint8, device=dev)
    for _ in range(5):
        out = a.sample_step(logits, actions=acts, log_probs=lp, entropy=ent, rewards=rew, dones=don)
        ref = b.sample_step(logits)
        assert out[0] is acts and out[1] is lp and out[2] is ent and out[3] is rew
        for x, y in zip(out, ref):
            assert torch.equal(x, y)
    with pytest.raises(ValueError):
        a.sample_step(logits, actions=torch.empty(E, dtype=torch.int64, device=dev))
    with pytest.raises(ValueError):
        a.sample_step(logits, log_probs=torch.empty(E - 1, device=dev))
    # outputs switched off: nothing returned for them, the step still happens
    ref = b.sample_step(logits)
    out = a.sample_step(logits, dones=False, rewards=False)
    assert out[3] is None and out[4] is None
    assert torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)
    # inputs a launch would read out of place are refused before it
    with pytest.raises(ValueError):
        a.sample_step(logits.cpu())
    with pytest.raises(ValueError):
        a.sample_actions(logits.cpu())
    with pytest.raises(ValueError):
        a.sample_step(logits, uniforms=torch.rand(E - 1, device=dev))
    with pytest.raises(ValueError):
        a.sample_actions(logits, uniforms=torch.rand(E - 1, device=dev))


@pytest.mark.parametrize("n_board,E", [(8, 2049), (8, 40000), (7, 40000), (6, 20000), (10, 5001)])
def test_sample_step_without_auto_reset(torch_gpu, n_board, E):
    """Every lane layout of oth_sample_step (quads up to 16,384 boards, pairs for
    7x7 / 8x8 beyond and for two-word boards, one lane otherwise) against sample_actions + step without
    auto-reset: games end and stay terminated with stale possible_moves, the
    sampler still draws on them, step answers done with reward 0
    (othello.py:415-416), both flag settings of the rewards."""
    torch = torch_gpu
    from gymothelloenv_amd import VecOthelloEnv
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(E + n_board)
    for disk in (False, True):
        kw = dict(board_size=n_board, auto_reset=False, num_disk_as_reward=disk, seed=5, device=dev)
        fused, split = VecOthelloEnv(E, **kw), VecOthelloEnv(E, **kw)
        fused.reset()
        split.reset()
        for k in range(n_board * n_board + 4):
            logits = torch.randn(E, n_board * n_board, device=dev, generator=g)
            uni = torch.rand(E, device=dev, generator=g)
            a1, lp1, en1, r1, d1 = fused.sample_step(logits, uniforms=uni)
            a2, lp2, en2 = split.sample_actions(logits, uniforms=uni)
            _, r2, d2, _ = split.step(a2, observe=False)
            assert torch.equal(a1, a2) and torch.equal(lp1, lp2) and torch.equal(en1, en2), k
            assert torch.equal(r1, r2) and torch.equal(d1, d2), k
        for x, y in zip(fused.get_state(), split.get_state()):
            assert torch.equal(x, y)
        assert bool(d1.all())  # every game over after N*N plies
        assert torch.equal(fused.counts(), split.counts())
