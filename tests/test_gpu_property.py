"""Property tests (hypothesis) of the device kernels on
ARBITRARY positions: random disjoint disc masks of any density, either side to
move, reachable in play or not (set_board_state, othello.py:380-389, accepts
any board), against the oracle restatement on the same positions:

  * get_possible_actions (othello.py:313-343) through the stateless entry point;
  * one step (othello.py:412-462) with legal, illegal and out-of-range actions,
    in both sudden-death modes and both reward modes, from boards where the
    mover (or both sides) may have no move;
  * the observation layouts (othello.py:257,363-376; util.py:48-74) and
    count_disks (:468-471);
  * GreedyPolicy and MaxiMin-2 / -3 (simple_policies.py:69-163);
  * multi-ply random and greedy play with auto-reset from such positions;
  * OthelloEnv.step on the device against random and greedy opponents;
  * the single-board record of oth_step_sync and the learners' fused ply.

Hypothesis draws the board size, the disc densities and the seed of the
position generator (derandomized: the same examples every run, no example
database written); each example checks a batch of 96 boards (one and a half
waves: a ragged last wave)."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import oracle

pytestmark = pytest.mark.gpu

E = 96
SIZES = [4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 16]
SETTINGS = dict(max_examples=60, deadline=None, derandomize=True, database=None,
                suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])

_ENVS = {}


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    yield torch
    for env in list(_ENVS.values()) + list(_PLAY.values()):
        env.close()
    _ENVS.clear()
    _PLAY.clear()


def _env(n, sd=True, disk=False):
    from gymothelloenv_amd import VecOthelloEnv
    key = (n, sd, disk)
    if key not in _ENVS:
        _ENVS[key] = VecOthelloEnv(E, board_size=n, sudden_death_on_invalid_move=sd, num_disk_as_reward=disk,
                                   auto_reset=False, seed=0, device="cuda:0")
    return _ENVS[key]


def _pack(mask, n):
    W = oracle.nwords(n)
    out = np.zeros((mask.shape[0], W), dtype=np.uint64)
    for a in range(n * n):
        out[:, a // 64] |= mask[:, a].astype(np.uint64) << np.uint64(a % 64)
    return out


def _positions(n, seed, db, dw):
    """E arbitrary positions: each square black with probability db, white with
    dw, else empty; the side to move drawn per board; possible_moves as the
    oracle computes them for that side."""
    rng = np.random.RandomState(seed)
    u = rng.rand(E, n * n)
    black, white = u < db, (u >= db) & (u < db + dw)
    B, Wt = _pack(black, n), _pack(white, n)
    turn = np.where(rng.rand(E) < 0.5, 1, -1)  # +1: white to move
    tw = (turn == 1)[:, None]
    s = oracle.State(n, E)
    s.boards[:] = np.concatenate([B, Wt], 1)
    s.meta[:] = oracle.meta_from(turn)
    s.legal[:] = oracle.legal(n, np.where(tw, Wt, B), np.where(tw, B, Wt))
    return s


def _load(torch, env, s):
    env.set_state(torch.from_numpy(s.boards.view(np.int64)), torch.from_numpy(s.meta.view(np.int16)),
                  torch.from_numpy(s.legal.view(np.int64)))


def _state_np(env):
    b, m, lg = env.get_state()
    return b.cpu().numpy().view(np.uint64), m.cpu().numpy().view(np.uint16), lg.cpu().numpy().view(np.uint64)


position = dict(n=st.sampled_from(SIZES), seed=st.integers(0, 2 ** 31 - 1),
                db=st.floats(0.0, 0.7), dw=st.floats(0.0, 0.7))


@settings(**SETTINGS)
@given(**position)
def test_legal_moves_on_arbitrary_positions(torch_cuda, n, seed, db, dw):
    torch = torch_cuda
    from gymothelloenv_amd.vec_env import legal_moves
    s = _positions(n, seed, db, min(dw, 1.0 - db))
    W = s.W
    mover = torch.from_numpy(s.boards[:, :W].view(np.int64)).cuda()
    opp = torch.from_numpy(s.boards[:, W:].view(np.int64)).cuda()
    got = legal_moves(n, mover, opp).cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got, oracle.legal(n, s.boards[:, :W], s.boards[:, W:]))


@settings(**SETTINGS)
@given(sd=st.booleans(), disk=st.booleans(), **position)
def test_step_on_arbitrary_positions(torch_cuda, n, seed, db, dw, sd, disk):
    torch = torch_cuda
    s = _positions(n, seed, db, min(dw, 1.0 - db))
    env = _env(n, sd, disk)
    _load(torch, env, s)
    rng = np.random.RandomState(seed ^ 0x5A5A)
    acts = rng.randint(0, n * n, size=E).astype(np.int32)  # mostly illegal squares
    for e in range(E):  # a third legal, a few out of range
        sq = [a for a in range(n * n) if (int(s.legal[e, a // 64]) >> (a % 64)) & 1]
        r = rng.rand()
        if sq and r < 0.34:
            acts[e] = sq[rng.randint(len(sq))]
        elif r > 0.94:
            acts[e] = -1 if r > 0.97 else n * n + 2
    flags = (oracle.F_SUDDEN_DEATH if sd else 0) | (oracle.F_DISK_REWARD if disk else 0)
    orw, od, _ = oracle.step(s, flags, acts, seed=0, ply=0)
    _, r, d, _ = env.step(torch.from_numpy(acts).cuda(), observe=False)
    np.testing.assert_array_equal(r.cpu().numpy(), orw)
    np.testing.assert_array_equal(d.cpu().numpy(), od.astype(bool))
    b, m, lg = _state_np(env)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)


@settings(**SETTINGS)
@given(**position)
def test_observations_and_counts_on_arbitrary_positions(torch_cuda, n, seed, db, dw):
    torch = torch_cuda
    s = _positions(n, seed, db, min(dw, 1.0 - db))
    env = _env(n)
    _load(torch, env, s)
    obs, obs2, ms = oracle.observe(s)
    for lay, want in (("board", obs), ("board_legal", obs2), ("make_state", ms)):
        for dt in (torch.int8, torch.float32, torch.int64):
            got = env.observe(lay, dt).cpu().numpy()
            np.testing.assert_array_equal(got, want.astype(got.dtype), err_msg="%s %s" % (lay, dt))
    np.testing.assert_array_equal(env.count_disks().cpu().numpy(), oracle.count_disks(s))


@settings(**SETTINGS)
@given(n=st.sampled_from([4, 5, 6, 7, 8, 9, 10]), seed=st.integers(0, 2 ** 31 - 1),
       db=st.floats(0.05, 0.5), dw=st.floats(0.05, 0.5))
def test_scripted_policies_on_arbitrary_positions(torch_cuda, n, seed, db, dw):
    torch = torch_cuda
    s = _positions(n, seed, db, min(dw, 1.0 - db))
    env = _env(n)
    _load(torch, env, s)
    np.testing.assert_array_equal(env.greedy_actions().cpu().numpy(), oracle.greedy(s))
    for depth in (2, 3):
        np.testing.assert_array_equal(env.policy_actions("maximin%d" % depth).cpu().numpy(),
                                      oracle.maximin(s, depth), err_msg="maximin%d" % depth)


_PLAY = {}


def _play_env(n, disk):
    from gymothelloenv_amd import VecOthelloEnv
    if (n, disk) not in _PLAY:
        _PLAY[(n, disk)] = VecOthelloEnv(E, board_size=n, num_disk_as_reward=disk, auto_reset=True, seed=77,
                                         device="cuda:0")
    return _PLAY[(n, disk)]


@settings(**SETTINGS)
@given(policy=st.sampled_from(["random", "greedy"]), disk=st.booleans(), plies=st.integers(1, 24), **position)
def test_play_from_arbitrary_positions(torch_cuda, n, seed, db, dw, policy, disk, plies):
    """The fused multi-ply kernels (k_play_rand / k_play_rand_w / k_play) from
    arbitrary positions -- boards whose mover or both sides have no move, which
    the fast path hands to the per-ply path -- with auto-reset: actions,
    rewards, dones, the final state and the W/D/L tally equal the oracle's
    rollout (the same Philox draws by global env id and ply)."""
    torch = torch_cuda
    s = _positions(n, seed, db, min(dw, 1.0 - db))
    env = _play_env(n, disk)
    _load(torch, env, s)
    ply0 = env.ply_counter
    env.counts(reset=True)
    a, r, d = env.step_policy(policy, n_plies=plies)
    flags = oracle.F_AUTO_RESET | oracle.F_SUDDEN_DEATH | (oracle.F_DISK_REWARD if disk else 0)
    oa, orw, od, owdl = oracle.rollout(s, flags, 0 if policy == "random" else 1, plies, seed=77, ply0=ply0)
    np.testing.assert_array_equal(a.cpu().numpy(), oa)
    np.testing.assert_array_equal(r.cpu().numpy(), orw)
    np.testing.assert_array_equal(d.cpu().numpy(), od)
    b, m, lg = _state_np(env)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)
    np.testing.assert_array_equal(env.counts().cpu().numpy(), owdl)


def _vs_env(n):
    from gymothelloenv_amd import VecOthelloEnv
    if ("vs", n) not in _PLAY:
        _PLAY[("vs", n)] = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=91, device="cuda:0")
    return _PLAY[("vs", n)]


@settings(**SETTINGS)
@given(opp=st.sampled_from(["random", "greedy"]), **position)
def test_step_vs_from_arbitrary_positions(torch_cuda, n, seed, db, dw, opp):
    """OthelloEnv.step on the device (oth_step_vs_observe: the protagonist's
    action, the device opponent's replies until the protagonist moves again,
    -reward after an opponent ply ended the game, auto-reset; othello.py:176-200)
    from arbitrary positions with the side to move as the protagonist, legal
    and illegal actions: rewards, dones, plies, state and the returned
    observation equal the oracle's."""
    torch = torch_cuda
    s = _positions(n, seed, db, min(dw, 1.0 - db))
    prot = np.where(s.meta & 1, 1, -1).astype(np.int8)
    env = _vs_env(n)
    _load(torch, env, s)
    call = env.ply_counter
    rng = np.random.RandomState(seed ^ 0x7777)
    acts = rng.randint(-1, n * n, size=E).astype(np.int32)
    for e in range(E):
        sq = [a for a in range(n * n) if (int(s.legal[e, a // 64]) >> (a % 64)) & 1]
        if sq and rng.rand() < 0.8:
            acts[e] = sq[rng.randint(len(sq))]
    o, r, d, pl = env.step_vs(torch.from_numpy(acts).cuda(), opponent=opp, protagonist=torch.from_numpy(prot).cuda(),
                              obs_layout="board")
    orw, od, opl = oracle.step_vs(s, oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET, 0 if opp == "random" else 1,
                                  call, acts, seed=91, prot=prot)
    np.testing.assert_array_equal(r.cpu().numpy(), orw)
    np.testing.assert_array_equal(d.cpu().numpy(), od.astype(bool))
    np.testing.assert_array_equal(pl.cpu().numpy(), opl)
    b, m, lg = _state_np(env)
    np.testing.assert_array_equal(b, s.boards)
    np.testing.assert_array_equal(m, s.meta)
    np.testing.assert_array_equal(lg, s.legal)
    np.testing.assert_array_equal(o.cpu().numpy(), oracle.observe(s)[0].astype(np.int64))


@settings(**SETTINGS)
@given(sd=st.booleans(), which=st.integers(0, E - 1), **position)
def test_step_sync_record_on_arbitrary_positions(torch_cuda, n, seed, db, dw, sd, which):
    """oth_step_sync (the drop-in's one launch per step(): the board stepped with
    a host action, then its whole record written into mapped host memory) on an
    arbitrary position: state, reward / done, count_disks, GreedyPolicy's move
    and both observation layouts equal the oracle's."""
    import ctypes

    from gymothelloenv_amd import _lib as L
    torch = torch_cuda
    s = _positions(n, seed, db, min(dw, 1.0 - db))
    env = _env(n, sd)
    _load(torch, env, s)
    one = oracle.State(n, 1)
    one.boards[:], one.meta[:], one.legal[:] = s.boards[which], s.meta[which], s.legal[which]
    nn, W = n * n, s.W
    rng = np.random.RandomState(seed ^ 0x1234)
    legal = [a for a in range(nn) if (int(one.legal[0, a // 64]) >> (a % 64)) & 1]
    a = int(rng.choice(legal)) if legal and rng.rand() < 0.7 else int(rng.randint(-2, nn + 2))
    orw, od, _ = oracle.step(one, oracle.F_SUDDEN_DEATH if sd else 0, np.array([a], dtype=np.int32))
    layout = L.OTH_OBS_BOARD_LEGAL if seed & 1 else L.OTH_OBS_BOARD
    ptr = ctypes.c_void_p()
    L.check(env._lib.oth_step_sync(env._h, which, 1 | L.OTH_RECORD_GREEDY, a, layout, ctypes.byref(ptr),
                                   env._stream()), "oth_step_sync")
    rec = L.OthRecord.from_address(ptr.value)
    assert list(rec.black)[:W] == list(one.boards[0, :W]) and list(rec.white)[:W] == list(one.boards[0, W:])
    assert list(rec.legal)[:W] == list(one.legal[0]) and rec.meta == one.meta[0]
    assert (rec.reward, rec.done) == (int(orw[0]), int(od[0]))
    wb = oracle.count_disks(one)[0]
    assert (rec.white_cnt, rec.black_cnt) == (wb[0], wb[1])
    if not one.meta[0] & 2:
        now = [x for x in range(nn) if (int(one.legal[0, x // 64]) >> (x % 64)) & 1]
        assert rec.greedy == (int(oracle.greedy(one)[0]) if now else -1)
    obs, obs2, _ = oracle.observe(one)
    got = np.ctypeslib.as_array(rec.obs)[:(2 if seed & 1 else 1) * nn]
    np.testing.assert_array_equal(got, (obs2 if seed & 1 else obs).reshape(-1))


@settings(**SETTINGS)
@given(lay=st.sampled_from(["board", "board_legal", "make_state"]), **position)
def test_sample_step_observe_on_arbitrary_positions(torch_cuda, n, seed, db, dw, lay):
    """The learners' fused ply (oth_sample_step_observe: masked sample, step and
    the next observation in one launch where the board is one word) from
    arbitrary positions -- including boards without a possible move (action 0,
    log-prob 0: model.py:69-71) -- equals sample_actions + step + observe on a
    twin handle, and the step and observation equal the oracle's."""
    torch = torch_cuda
    s = _positions(n, seed, db, min(dw, 1.0 - db))
    fused = _env(n)
    twin = _ENVS.setdefault((n, "twin"), None)  # a second handle with the same flags and seed
    if twin is None:
        from gymothelloenv_amd import VecOthelloEnv
        twin = _ENVS[(n, "twin")] = VecOthelloEnv(E, board_size=n, auto_reset=False, seed=0, device="cuda:0")
    _load(torch, fused, s)
    _load(torch, twin, s)
    fused.sample_counter = twin.sample_counter = 0
    g = torch.Generator(device="cuda").manual_seed(seed)
    logits = torch.randn(E, n * n, device="cuda", generator=g) * 2
    a1, lp1, en1, r1, d1, o1 = fused.sample_step(logits, observe=lay, obs_dtype=torch.float32)
    a2, lp2, en2 = twin.sample_actions(logits)
    _, r2, d2, _ = twin.step(a2, observe=False)
    o2 = twin.observe(lay, torch.float32)
    assert torch.equal(a1, a2) and torch.equal(lp1, lp2) and torch.equal(en1, en2)
    assert torch.equal(r1, r2) and torch.equal(d1, d2) and torch.equal(o1, o2)
    orw, od, _ = oracle.step(s, oracle.F_SUDDEN_DEATH, a1.cpu().numpy())
    np.testing.assert_array_equal(r1.cpu().numpy(), orw)
    obs, obs2, ms = oracle.observe(s)
    want = {"board": obs, "board_legal": obs2, "make_state": ms}[lay]
    np.testing.assert_array_equal(o1.cpu().numpy(), want.astype(np.float32))
