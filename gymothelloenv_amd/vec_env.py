"""VecOthelloEnv -- E Othello boards resident in HBM, stepped by HIP kernels.

The batched form of the reference's OthelloBaseEnv (othello.py:217-501): one
handle of the C ABI (include/othello_mi355x.h) owns E boards on one GPU; every
method enqueues kernels on the current torch stream and returns torch tensors
that stay on the device.  It replaces the reference's CPU "vector env" of one
process per board (envs.py:7-287) for the hot path; torch here is only device
memory, streams and the collective for the W/D/L tally.
"""
import contextlib
import ctypes

import torch

from . import _lib as L
from .masked import _rows

_OBS_LAYOUTS = {"board": L.OTH_OBS_BOARD, "board_legal": L.OTH_OBS_BOARD_LEGAL,
                "make_state": L.OTH_OBS_MAKE_STATE, "absolute": L.OTH_OBS_ABSOLUTE, "legal": L.OTH_OBS_LEGAL}
_OBS_PLANES = {L.OTH_OBS_BOARD: 1, L.OTH_OBS_BOARD_LEGAL: 2, L.OTH_OBS_MAKE_STATE: 4, L.OTH_OBS_ABSOLUTE: 1,
               L.OTH_OBS_LEGAL: 1}
_ONE_PLANE = (L.OTH_OBS_BOARD, L.OTH_OBS_ABSOLUTE, L.OTH_OBS_LEGAL)
_DTYPES = {torch.int8: L.OTH_I8, torch.int32: L.OTH_I32, torch.int64: L.OTH_I64,
           torch.float32: L.OTH_F32, torch.float64: L.OTH_F64, torch.bfloat16: L.OTH_BF16}
_POLICIES = {"random": L.OTH_POLICY_RANDOM, "greedy": L.OTH_POLICY_GREEDY}
_POLICIES.update({"maximin%d" % d: L.OTH_POLICY_MAXIMIN(d) for d in range(1, L.OTH_MAXIMIN_MAX_DEPTH + 1)})

BLACK_DISK, NO_DISK, WHITE_DISK = -1, 0, 1  # othello.py:10-12


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def nwords(n):
    return (n * n + 63) // 64


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class VecOthelloEnv(object):
    """E independent boards of one size on one GPU.

    Args mirror OthelloBaseEnv / SimpleOthelloEnv (othello.py:26-33, 222-227);
    the batched extras are `auto_reset` (reset a board right after its terminal
    ply), `seed` / `env_id_base` (Philox key and this shard's first global env
    id) and `device`.
    """

    def __init__(self, num_envs, board_size=8, sudden_death_on_invalid_move=True,
                 num_disk_as_reward=False, possible_actions_in_obs=False, auto_reset=False,
                 initial_rand_steps=0, seed=0, env_id_base=0, device=None, lib=None):
        self._lib = lib if lib is not None else L.load()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:  # "cuda" -> the current device, by index
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.num_envs = int(num_envs)
        self.board_size = max(4, int(board_size))  # othello.py:230
        self.words = nwords(self.board_size)
        self.sudden_death_on_invalid_move = bool(sudden_death_on_invalid_move)
        self.num_disk_as_reward = bool(num_disk_as_reward)
        self.possible_actions_in_obs = bool(possible_actions_in_obs)
        self.auto_reset = bool(auto_reset)
        self.initial_rand_steps = int(initial_rand_steps)
        self.seed = int(seed)
        self.env_id_base = int(env_id_base)
        flags = ((L.OTH_SUDDEN_DEATH if self.sudden_death_on_invalid_move else 0) |
                 (L.OTH_DISK_REWARD if self.num_disk_as_reward else 0) |
                 (L.OTH_AUTO_RESET if self.auto_reset else 0))
        self.flags = flags
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            L.check(self._lib.oth_create(self.num_envs, self.board_size, flags, self.seed & (2 ** 64 - 1),
                                         self.env_id_base, self.initial_rand_steps, self.device.index,
                                         ctypes.byref(h)), "oth_create")
        self._h = h
        self._hv = h.value  # the handle as an int: the per-step ctypes calls take it as is
        self._dev_index = self.device.index
        self._step_fn = self._lib.oth_step
        self._step_obs_fn = self._lib.oth_step_observe
        self._bview = None  # (dones tensor, its bool view): step()'s view of caller-given dones, cached
        self._okbufs = None  # (rewards, dones) tensors step() has checked
        self._okobs = None  # (obs tensor, layout) step() / sample_step() have checked
        self._sample_calls = 0  # Philox counter of sample_actions
        self._region_resets = None  # resets inside an open graph region (None: no region)

    # ------------------------------------------------------------------ utils
    def _stream(self):
        if _RAW_STREAM is not None:  # the current stream's handle without building a Stream object
            return ctypes.c_void_p(_RAW_STREAM(self.device.index))
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.oth_destroy(self._h)
            self._h = None
            self._hv = None  # a later step() passes NULL: OTH_EINVAL, not a freed handle

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _i32(self, *shape):
        return torch.empty(*shape, dtype=torch.int32, device=self.device)

    def _u8(self, *shape):
        return torch.empty(*shape, dtype=torch.uint8, device=self.device)

    def _out(self, given, dtype, name):
        """An (E,) output: a new tensor for None / True, nothing for False, or the
        caller's tensor (checked) to be written in place."""
        if given is None or given is True:
            return torch.empty(self.num_envs, dtype=dtype, device=self.device)
        if given is False:
            return None
        if given.dtype != dtype or given.numel() != self.num_envs or not given.is_contiguous() or \
                given.device != self.device:
            raise ValueError("%s must be a contiguous %s tensor of %d elements on %s" %
                             (name, dtype, self.num_envs, self.device))
        return given

    @property
    def ply_counter(self):
        return int(self._lib.oth_ply_counter(self._h))

    @ply_counter.setter
    def ply_counter(self, v):
        if getattr(self, "_region_resets", None) is not None:
            raise RuntimeError("cannot set the ply counter inside a graph region")
        L.check(self._lib.oth_set_ply_counter(self._h, int(v)), "oth_set_ply_counter")

    # ---------------------------------------------------------------- the API
    def reset(self, mask=None):
        """OthelloBaseEnv.reset (othello.py:265-271) for every board (or where mask)."""
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        if getattr(self, "_region_resets", None) is not None:
            self._region_resets += 1
        L.check(self._lib.oth_reset(self._h, _ptr(m), self._stream()), "oth_reset")
        return self.get_observation()

    def step(self, actions, rewards=None, dones=None, observe=True, obs=None, obs_layout=None,
             obs_dtype=torch.int64):
        """OthelloBaseEnv.step (othello.py:412-462) on every board.

        actions: int tensor (E,).  rewards / dones: optional int32 / uint8 (or
        bool) (E,) tensors on this device, written in place (the loop form: no
        allocation per step; checked once per tensor).  Returns (obs, rewards
        int32 (E,), dones bool (E,), None).  With observe (the default) obs is the
        step's get_observation() (othello.py:462) -- or `obs_layout` ('board',
        'board_legal', 'make_state', 'absolute', 'legal') -- written by the same
        launch that stepped the boards (oth_step_observe), into `obs` if given (its
        dtype decides the element type) or a new `obs_dtype` tensor; None when
        observe=False.  The host path is one ctypes call: an int32 contiguous
        action tensor on this device is passed as is."""
        a = actions
        if a.dtype is not torch.int32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.int32).contiguous()
        if a.numel() != self.num_envs:
            raise ValueError("expected %d actions, got %d" % (self.num_envs, a.numel()))
        r = rewards if rewards is not None else self._i32(self.num_envs)
        d = dones if dones is not None else self._u8(self.num_envs)
        ok = self._okbufs
        # caller-given buffers: checked once each, and again if resize_() / set_() moved or shrank them
        if ok is None or ok[0] is not r or ok[1] is not d or ok[2] != (r.data_ptr(), d.data_ptr(), r.numel(),
                                                                      d.numel()):
            self._check_out(r, (torch.int32,), "rewards")
            self._check_out(d, (torch.uint8, torch.bool), "dones")
            self._okbufs = (r, d, (r.data_ptr(), d.data_ptr(), r.numel(), d.numel()))
        st = _RAW_STREAM(self._dev_index) if _RAW_STREAM is not None else self._stream()
        if observe:
            lay, o = self._obs_out(obs_layout, obs_dtype, obs)
            rc = self._step_obs_fn(self._hv, a.data_ptr(), r.data_ptr(), d.data_ptr(), lay, _DTYPES[o.dtype],
                                   o.data_ptr(), st)
            if rc:
                L.check(rc, "oth_step_observe")
        else:
            o = None
            rc = self._step_fn(self._hv, a.data_ptr(), r.data_ptr(), d.data_ptr(), st)
            if rc:
                L.check(rc, "oth_step")
        bv = self._bview
        if bv is None or bv[0] is not d:  # 0/1 bytes: a view, not a conversion kernel
            bv = self._bview = (d, d if d.dtype is torch.bool else d.view(torch.bool))
        return o, r, bv[1], None

    def _check_out(self, t, dtypes, name):
        """A caller-given (E,) output the kernels write: on this device, contiguous,
        E elements of one of `dtypes` -- else ValueError before any launch."""
        if not isinstance(t, torch.Tensor) or t.dtype not in dtypes or t.device != self.device or \
                not t.is_contiguous() or t.numel() != self.num_envs:
            raise ValueError("%s must be a contiguous %s tensor of %d elements on %s" %
                             (name, " or ".join(str(x) for x in dtypes), self.num_envs, self.device))

    def _obs_shape(self, lay):
        n = self.board_size
        return (self.num_envs, n, n) if lay in _ONE_PLANE else (self.num_envs, _OBS_PLANES[lay], n, n)

    def _obs_out(self, layout, dtype, out):
        """(layout id, output tensor) of a fused observation: get_observation()'s
        layout unless given; `out` checked once per tensor, or a new tensor."""
        if layout is None:
            lay = L.OTH_OBS_BOARD_LEGAL if self.possible_actions_in_obs else L.OTH_OBS_BOARD
        else:
            lay = _OBS_LAYOUTS[layout] if isinstance(layout, str) else int(layout)
            if lay not in _OBS_PLANES:
                raise ValueError("unknown observation layout %r" % (layout,))
        if out is None:
            if dtype not in _DTYPES:
                raise ValueError("observation dtype must be one of %s" % list(_DTYPES))
            return lay, torch.empty(self._obs_shape(lay), dtype=dtype, device=self.device)
        ok = self._okobs
        if ok is None or ok[0] is not out or ok[1] != lay or ok[2] != (out.data_ptr(), out.numel(), out.dtype):
            shape = self._obs_shape(lay)
            if out.dtype not in _DTYPES or out.device != self.device or not out.is_contiguous() or \
                    out.numel() != _numel(shape):
                raise ValueError("obs must be a contiguous tensor of %s elements (shape %s) of one of %s on %s" %
                                 (_numel(shape), shape, list(_DTYPES), self.device))
            self._okobs = (out, lay, (out.data_ptr(), out.numel(), out.dtype))
        return lay, out

    def step_policy(self, policy="random", n_plies=1, actions=None, rewards=None, dones=None, record=True):
        """n_plies plies where every board's mover plays `policy` on the device
        (RandomPolicy simple_policies.py:37-41, GreedyPolicy :69-92, MaxiMinPolicy
        :98-163 as 'maximin1'..'maximin10').

        Returns (actions, rewards, dones) of shape (n_plies, E) (None if not recorded)."""
        pol = _POLICIES[policy] if isinstance(policy, str) else int(policy)
        if record:
            actions = actions if actions is not None else self._i32(n_plies, self.num_envs)
            rewards = rewards if rewards is not None else self._i32(n_plies, self.num_envs)
            dones = dones if dones is not None else self._u8(n_plies, self.num_envs)
        L.check(self._lib.oth_step_policy(self._h, pol, int(n_plies), _ptr(actions), _ptr(rewards),
                                          _ptr(dones), self._stream()), "oth_step_policy")
        return actions, rewards, dones

    # ------------------------------------------- OthelloEnv semantics on device
    def _protagonist(self, protagonist):
        if protagonist is None:
            return getattr(self, "_prot", None)
        if isinstance(protagonist, int):
            protagonist = torch.full((self.num_envs,), protagonist, dtype=torch.int8)
        t = protagonist.to(device=self.device, dtype=torch.int8).contiguous()
        if t.numel() != self.num_envs:
            raise ValueError("protagonist needs one colour per board")
        self._prot = t
        return t

    def reset_vs(self, opponent="random", protagonist=None, mask=None):
        """OthelloEnv.reset (othello.py:151-174) for every board: reset, then the
        embedded opponent (`opponent` = 'random' | 'greedy', played on the device)
        replies until the protagonist (+1 white, the reference default, or -1
        black; int or per-board tensor) is to move."""
        prot = self._protagonist(protagonist)
        m = None if mask is None else mask.to(device=self.device, dtype=torch.uint8).contiguous()
        L.check(self._lib.oth_reset_vs(self._h, _POLICIES[opponent], _ptr(prot), _ptr(m), self._stream()),
                "oth_reset_vs")
        return self.get_observation()

    def step_vs(self, actions, opponent="random", protagonist=None, observe=True, obs=None, obs_layout=None,
                obs_dtype=torch.int64):
        """OthelloEnv.step (othello.py:176-200) for every board: the protagonist
        plays `actions`, the device opponent replies until the protagonist is to
        move again.  Returns (obs, rewards (protagonist's view, negated after an
        opponent ply ended the game), dones bool, plies applied per board).  The
        observation (get_observation's layout unless `obs_layout`; into `obs` if
        given) comes from the same launch (oth_step_vs_observe)."""
        prot = self._protagonist(protagonist)
        a = actions.to(device=self.device, dtype=torch.int32).contiguous()
        if a.numel() != self.num_envs:
            raise ValueError("expected %d actions, got %d" % (self.num_envs, a.numel()))
        r, d, n = self._i32(self.num_envs), self._u8(self.num_envs), self._i32(self.num_envs)
        if observe:
            lay, o = self._obs_out(obs_layout, obs_dtype, obs)
            L.check(self._lib.oth_step_vs_observe(self._h, _POLICIES[opponent], _ptr(a), _ptr(prot), _ptr(r),
                                                  _ptr(d), _ptr(n), lay, _DTYPES[o.dtype], _ptr(o), self._stream()),
                    "oth_step_vs_observe")
        else:
            o = None
            L.check(self._lib.oth_step_vs(self._h, _POLICIES[opponent], _ptr(a), _ptr(prot), _ptr(r), _ptr(d),
                                          _ptr(n), self._stream()), "oth_step_vs")
        return o, r, d.view(torch.bool), n

    def legal_mask(self):
        """possible_moves of every board as (E, W) int64 bit masks (bit a = square a)."""
        out = torch.empty(self.num_envs, self.words, dtype=torch.int64, device=self.device)
        L.check(self._lib.oth_legal(self._h, _ptr(out), self._stream()), "oth_legal")
        return out

    def legal_actions(self):
        """possible_moves as a bool (E, N*N) tensor: the OTH_OBS_LEGAL plane in int8,
        viewed as bool (one kernel writing E*N*N bytes, no conversion)."""
        o = self.observe("legal", torch.int8)
        return o.view(torch.bool).reshape(self.num_envs, -1)

    def greedy_actions(self):
        """GreedyPolicy.get_action (simple_policies.py:69-92) for every board."""
        return self.policy_actions("greedy")

    def policy_actions(self, policy="greedy"):
        """The move of a scripted policy ('greedy', 'maximin<d>'; simple_policies.py:57-163)
        for the side to move on every board.

        MaxiMin accepts any depth, as the reference does (:101-103).  Every search
        level places a disc, so a search deeper than a board's empty squares is the
        search of depth = its empty squares (the board is full, hence terminal, at
        that level either way, :117-126).  Beyond OTH_MAXIMIN_MAX_DEPTH the call
        therefore runs at the largest empty-square count of the batch's live
        boards when that is at most OTH_MAXIMIN_MAX_DEPTH (bit-identical), and
        raises otherwise.  Depth <= 0 searches nothing: the reference's search
        stops at the root and returns no move (:117-126), so every board gets -1.
        Calls the C ABI estimates above OTH_MAXIMIN_LEAF_BUDGET leaves (bounded by
        each board's empty squares) raise OthelloLibError."""
        if isinstance(policy, str) and policy.startswith("maximin") and policy not in _POLICIES:
            try:
                d = int(policy[len("maximin"):])
            except ValueError:
                raise ValueError("unknown policy %r: 'greedy' or 'maximin<depth>'" % (policy,)) from None
            if d <= 0:
                return torch.full((self.num_envs,), -1, dtype=torch.int32, device=self.device)
            # (a terminated board's search returns no move at the root, whatever the depth)
            live = ~self.terminated()
            left = self.board_size ** 2 - self.count_disks().sum(1)
            empties = int(left[live].max()) if bool(live.any()) else 0
            if empties > L.OTH_MAXIMIN_MAX_DEPTH:
                raise ValueError("maximin%d: a board has %d empty squares; the device search covers depths up to "
                                 "%d, or any depth once every board has at most %d empty squares"
                                 % (d, empties, L.OTH_MAXIMIN_MAX_DEPTH, L.OTH_MAXIMIN_MAX_DEPTH))
            policy = "maximin%d" % max(1, min(d, empties))
        if isinstance(policy, str) and policy not in _POLICIES:
            raise ValueError("unknown policy %r: 'greedy' or 'maximin<depth>'" % (policy,))
        out = self._i32(self.num_envs)
        L.check(self._lib.oth_policy_actions(self._h, _POLICIES[policy], _ptr(out), self._stream()),
                "oth_policy_actions")
        return out

    def observe(self, layout="board", dtype=torch.int64, out=None):
        lay = _OBS_LAYOUTS[layout] if isinstance(layout, str) else int(layout)
        planes = _OBS_PLANES[lay]
        n = self.board_size
        shape = (self.num_envs, n, n) if lay in _ONE_PLANE else (self.num_envs, planes, n, n)
        if out is None:
            out = torch.empty(shape, dtype=dtype, device=self.device)
        L.check(self._lib.oth_observe(self._h, lay, _DTYPES[out.dtype], _ptr(out), self._stream()),
                "oth_observe")
        return out

    def get_observation(self, dtype=torch.int64):
        """get_observation (othello.py:363-378): mover-perspective board, plus the
        possible-moves plane when possible_actions_in_obs."""
        return self.observe("board_legal" if self.possible_actions_in_obs else "board", dtype)

    def make_state(self, dtype=torch.float32):
        """util.make_state (util.py:48-74) for every board: (E, 4, N, N)."""
        return self.observe("make_state", dtype)

    def count_disks(self):
        """count_disks (othello.py:468-471): int32 (E, 2) = (white_cnt, black_cnt)."""
        out = self._i32(self.num_envs, 2)
        L.check(self._lib.oth_count_disks(self._h, _ptr(out), self._stream()), "oth_count_disks")
        return out

    def set_player_turn(self, turn, mask=None):
        """set_player_turn (othello.py:464-466): set the turn and recompute possible_moves."""
        m = None if mask is None else mask.to(device=self.device, dtype=torch.uint8).contiguous()
        L.check(self._lib.oth_set_player_turn(self._h, int(turn), _ptr(m), self._stream()),
                "oth_set_player_turn")

    def get_state(self):
        """(boards (E, 2W) int64, meta (E,) int16, legal (E, W) int64) device copies
        in the exchange format of include/othello_mi355x.h."""
        b = torch.empty(self.num_envs, 2 * self.words, dtype=torch.int64, device=self.device)
        m = torch.empty(self.num_envs, dtype=torch.int16, device=self.device)
        lg = torch.empty(self.num_envs, self.words, dtype=torch.int64, device=self.device)
        L.check(self._lib.oth_get_state(self._h, _ptr(b), _ptr(m), _ptr(lg), self._stream()), "oth_get_state")
        return b, m, lg

    def set_state(self, boards=None, meta=None, legal=None):
        def dev(t, dt):
            return None if t is None else t.to(device=self.device).contiguous().view(dt)
        b, m, lg = dev(boards, torch.int64), dev(meta, torch.int16), dev(legal, torch.int64)
        for t, per in ((b, 2 * self.words), (m, 1), (lg, self.words)):
            if t is not None and t.numel() != self.num_envs * per:
                raise ValueError("state tensor has %d elements, expected %d" % (t.numel(), self.num_envs * per))
        L.check(self._lib.oth_set_state(self._h, _ptr(b), _ptr(m), _ptr(lg), self._stream()), "oth_set_state")
        # keep the sources alive until the async copies ran
        torch.cuda.current_stream(self.device).synchronize()

    def counts(self, reset=False):
        """{black wins, draws, white wins} of games finished since the last reset (int64 (3,))."""
        out = torch.empty(3, dtype=torch.int64, device=self.device)
        L.check(self._lib.oth_counts(self._h, _ptr(out), int(bool(reset)), self._stream()), "oth_counts")
        return out

    def counts_vs(self, reset=False):
        """{protagonist wins, draws, protagonist losses} of games finished by
        step_vs (run.py:100-130's count, the README's table) as int64 (3,)."""
        out = torch.empty(3, dtype=torch.int64, device=self.device)
        L.check(self._lib.oth_counts_vs(self._h, _ptr(out), int(bool(reset)), self._stream()), "oth_counts_vs")
        return out

    def _sampler_inputs(self, logits, uniforms):
        """(logits rows, uniforms) checked before a launch reads them: the rows on
        this handle's device, one per board; uniforms float32 on it, >= E of them."""
        x = _rows(logits, self.board_size)
        if x.device != self.device:
            raise ValueError("logits must be on %s (got %s)" % (self.device, x.device))
        if x.shape[0] != self.num_envs:
            raise ValueError("logits must have one row per board")
        if uniforms is not None:
            if uniforms.dtype != torch.float32 or not uniforms.is_contiguous() or uniforms.device != self.device:
                uniforms = uniforms.to(device=self.device, dtype=torch.float32).contiguous()
            if uniforms.numel() < self.num_envs:
                raise ValueError("uniforms must hold one value per board (%d), got %d" %
                                 (self.num_envs, uniforms.numel()))
        return x, uniforms

    def sample_actions(self, logits, deterministic=False, uniforms=None, log_probs=True, entropy=True):
        """Policy.act (model.py:60-99) for every board at once: sample (or, when
        deterministic, take the mode of) the softmax of `logits` (E, N*N)
        float32 restricted to the board's possible_moves.  Draws are Philox
        keyed (seed, env id, call counter) unless `uniforms` (E,) is given.
        Returns (actions int32, log_probs, entropy) on the device; the actions
        feed step() directly."""
        x, uniforms = self._sampler_inputs(logits, uniforms)
        acts = self._i32(self.num_envs)
        lp = torch.empty(self.num_envs, dtype=torch.float32, device=self.device) if log_probs else None
        ent = torch.empty(self.num_envs, dtype=torch.float32, device=self.device) if entropy else None
        mode = L.OTH_MASKED_MODE if deterministic else L.OTH_MASKED_SAMPLE
        L.check(self._lib.oth_sample_actions(self._h, _ptr(x), x.stride(0), _ptr(uniforms), self._sample_calls,
                                             mode, _ptr(acts), _ptr(lp), _ptr(ent), self._stream()),
                "oth_sample_actions")
        self._sample_calls += 1
        return acts, lp, ent

    def sample_step(self, logits, deterministic=False, uniforms=None, log_probs=True, entropy=True,
                    full_entropy=False, rewards=None, dones=None, actions=None, observe=None, obs=None,
                    obs_dtype=torch.float32):
        """sample_actions(logits) then step(actions) in ONE launch (oth_sample_step):
        Policy.act (model.py:60-99) over every board's possible_moves followed by
        OthelloBaseEnv.step (othello.py:412-462), bit-identical to the two calls.
        Returns (actions int32, log_probs, entropy, rewards int32, dones bool).
        Outputs may be given to be written in place: `actions` / `rewards` int32 (E,),
        `dones` uint8 (E,), and `log_probs` / `entropy` as float32 (E,) tensors
        instead of True.  observe: an observation layout ('make_state', the
        learners' next input (util.py:48-74), 'board', ...): the stepped boards'
        observation from the same launch (oth_sample_step_observe), into `obs` if
        given or a new `obs_dtype` tensor, appended as a sixth value."""
        x, uniforms = self._sampler_inputs(logits, uniforms)
        acts = self._out(actions, torch.int32, "actions")
        lp = self._out(log_probs, torch.float32, "log_probs")
        ent = self._out(entropy, torch.float32, "entropy")
        r = self._out(rewards, torch.int32, "rewards")
        d = self._out(dones, torch.uint8, "dones")
        mode = (L.OTH_MASKED_MODE if deterministic else L.OTH_MASKED_SAMPLE) | \
            (L.OTH_MASKED_FULL_ENTROPY if full_entropy else 0)
        if observe is None:
            L.check(self._lib.oth_sample_step(self._h, _ptr(x), x.stride(0), _ptr(uniforms), self._sample_calls,
                                              mode, _ptr(acts), _ptr(lp), _ptr(ent), _ptr(r), _ptr(d),
                                              self._stream()), "oth_sample_step")
        else:
            lay, o = self._obs_out(observe, obs_dtype, obs)
            L.check(self._lib.oth_sample_step_observe(self._h, _ptr(x), x.stride(0), _ptr(uniforms),
                                                      self._sample_calls, mode, _ptr(acts), _ptr(lp), _ptr(ent),
                                                      _ptr(r), _ptr(d), lay, _DTYPES[o.dtype], _ptr(o),
                                                      self._stream()), "oth_sample_step_observe")
        self._sample_calls += 1
        res = (acts, lp, ent, r, (d.view(torch.bool) if d is not None else None))
        return res if observe is None else res + (o,)

    @property
    def sample_counter(self):
        """Philox counter of the next eager sample_actions call (purpose 3)."""
        return self._sample_calls

    @sample_counter.setter
    def sample_counter(self, v):
        self._sample_calls = int(v)

    @staticmethod
    def graph_counter_base(slot):
        """First counter of graph region `slot`'s range (ply and sample counters)."""
        return int(slot) << L.OTH_GRAPH_COUNTER_SHIFT

    def graph_offsets(self, slot):
        """(ply, sample) offsets graph region `slot`'s replays have consumed;
        synchronises the device, so never call it during a capture."""
        _no_capture("graph_offsets")
        out = (ctypes.c_uint64 * 2)()
        L.check(self._lib.oth_graph_offsets(self._h, int(slot), out), "oth_graph_offsets")
        return int(out[0]), int(out[1])

    @contextlib.contextmanager
    def graph_region(self):
        """Wrap the calls captured into a HIP graph (enter it INSIDE
        `torch.cuda.graph`).  The region owns a counter range of its own
        (oth_graph_begin: ply and sample counters from slot << 40), and on exit
        enqueues the advance of its device offsets by what the region consumed,
        so replay r draws counters base + r*d .. base + r*d + d - 1: fresh
        Philox numbers every replay (random openings, device opponents,
        sample_actions without uniforms), disjoint from eager calls and from
        every other region of this handle.  Yields the slot.  A region that
        fails gives its slot back; a captured graph keeps it until
        release_graph_slot(slot) (call it when the graph is dropped).

            with torch.cuda.graph(g), env.graph_region() as slot:
                for k in range(K): env.step(env.sample_actions(actor(obs))[0]); ...
        """
        if not torch.cuda.is_current_stream_capturing():
            raise RuntimeError("graph_region must be entered inside torch.cuda.graph(...) "
                               "(with torch.cuda.graph(g), env.graph_region(): ...)")
        slot = ctypes.c_int32()
        L.check(self._lib.oth_graph_begin(self._h, ctypes.byref(slot)), "oth_graph_begin")
        k = int(slot.value)
        smp0, self._sample_calls = self._sample_calls, self.graph_counter_base(k)
        self._region_resets = 0
        ok = False
        try:
            yield k
            ok = True
        finally:
            capturing = torch.cuda.is_current_stream_capturing()
            d_smp = self._sample_calls - self.graph_counter_base(k)
            self._sample_calls = smp0
            d_ply = ctypes.c_uint64()
            rc = self._lib.oth_graph_end(self._h, d_smp, int(capturing), ctypes.byref(d_ply), self._stream())
            resets, self._region_resets = self._region_resets, None
            try:
                if ok:
                    L.check(rc, "oth_graph_end")
                    if not capturing:
                        raise RuntimeError("the capture ended inside graph_region: enter graph_region inside "
                                           "torch.cuda.graph(...), not around it")
                    if resets and self.initial_rand_steps > 0 and d_ply.value == 0:
                        raise RuntimeError("this graph region only resets boards with random openings: every "
                                           "replay would draw the same openings; capture at least one ply with "
                                           "the reset")
            except BaseException:
                ok = False
                raise
            finally:
                if not ok:  # no usable graph: the slot goes back
                    self._lib.oth_graph_release(self._h, k)

    def release_graph_slot(self, slot):
        """Give a graph region's counter slot back once its graph is dropped
        (oth_graph_release); the slot's offsets are kept, so a later region on
        it still draws counters no earlier replay drew."""
        L.check(self._lib.oth_graph_release(self._h, int(slot)), "oth_graph_release")

    def state_dict(self):
        """Boards, meta, possible_moves and the eager counters (host values).
        Graph regions keep their own counter ranges and are not part of it."""
        _no_capture("state_dict")
        b, m, lg = self.get_state()
        return {"boards": b, "meta": m, "legal": lg, "ply_counter": self.ply_counter,
                "sample_calls": self._sample_calls, "board_size": self.board_size,
                "num_envs": self.num_envs}

    def load_state_dict(self, sd):
        """Restore a state_dict.  Graphs captured on this handle stay valid and
        keep drawing from their own counter ranges (nothing is zeroed)."""
        _no_capture("load_state_dict")
        if sd["board_size"] != self.board_size or sd["num_envs"] != self.num_envs:
            raise ValueError("state_dict shape does not match this env")
        self.set_state(sd["boards"], sd["meta"], sd["legal"])
        self.ply_counter = sd["ply_counter"]
        self._sample_calls = int(sd.get("sample_calls", 0))

    # decoded views of the meta word
    def player_turn(self):
        b, m, _ = self.get_state()
        return torch.where((m & 1) != 0, WHITE_DISK, BLACK_DISK)

    def terminated(self):
        _, m, _ = self.get_state()
        return ((m >> 1) & 1) != 0

    def winner(self):
        _, m, _ = self.get_state()
        w = (m >> 2) & 3
        return torch.where(w == 1, WHITE_DISK, torch.where(w == 2, BLACK_DISK, NO_DISK))


def _numel(shape):
    k = 1
    for x in shape:
        k *= x
    return k


def _no_capture(what):
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("%s synchronises the device and cannot run during a HIP-graph capture" % what)


def legal_moves(board_size, mover, opponent):
    """Stateless get_possible_actions(board) (othello.py:313-343) on canonical
    boards given as (n, W) int64 mover / opponent masks on a GPU."""
    lib = L.load()
    mover = mover.contiguous()
    opponent = opponent.to(mover.device).contiguous()
    out = torch.empty_like(mover)
    stream = ctypes.c_void_p(torch.cuda.current_stream(mover.device).cuda_stream)
    L.check(lib.oth_legal_moves(int(board_size), int(mover.shape[0]), _ptr(mover), _ptr(opponent), _ptr(out),
                                stream), "oth_legal_moves")
    return out
