"""Drop-in OthelloBaseEnv / SimpleOthelloEnv / OthelloEnv backed by the HIP engine.

Same constructor arguments, attributes, methods and 4-tuple step returns as the
reference's othello.py, so its callers (ppo.py, simple_policies.py, the
harness workers) run unchanged.  Every rule decision -- legal moves, flips,
passes, terminal and reward, observations, disc counts -- is computed by the
kernels in csrc/ on a one-board VecOthelloEnv; the host only keeps a mirror
of the last device state (one packed device->host copy per synchronising
call) and converts it into the reference's Python types (lists, int64 boards).
The wrappers (SimpleOthelloEnv, OthelloEnv) are the reference's host-side
control flow around that engine, with the same np.random.RandomState calls
in the same order, so seeded runs reproduce the reference's trajectories.
"""
import numpy as np
import torch

from . import _lib as L
from .spaces import Box, Discrete
from .vec_env import VecOthelloEnv, legal_moves, nwords

BLACK_DISK = -1  # othello.py:10-12
NO_DISK = 0
WHITE_DISK = 1


def _mask_to_list(words, nn):
    out = []
    for wi, w in enumerate(words):
        w = int(w) & 0xFFFFFFFFFFFFFFFF
        while w:
            low = w & -w
            a = 64 * wi + low.bit_length() - 1
            if a < nn:
                out.append(a)
            w ^= low
    return out


def _list_to_mask(moves, n):
    W = nwords(n)
    words = [0] * W
    for a in moves:
        a = int(a)
        if 0 <= a < n * n:
            words[a // 64] |= 1 << (a % 64)
    return np.array([w if w < 2 ** 63 else w - 2 ** 64 for w in words], dtype=np.int64)


def _board_to_masks(board, n):
    """int board (N,N) with +1 / -1 / 0 -> (plus mask, minus mask) as int64 words."""
    flat = np.asarray(board).reshape(-1)
    if flat.size != n * n:
        raise ValueError("board has %d cells, expected %d" % (flat.size, n * n))
    return _list_to_mask(np.flatnonzero(flat == 1), n), _list_to_mask(np.flatnonzero(flat == -1), n)


class OthelloBaseEnv(object):
    """OthelloBaseEnv (othello.py:217-501) on one board in HBM."""

    metadata = {'render.modes': ['np_array', 'human']}

    def __init__(self, board_size=8, sudden_death_on_invalid_move=True, num_disk_as_reward=False,
                 possible_actions_in_obs=False, mute=False, device=None):
        self.board_size = max(4, board_size)  # othello.py:230
        self.sudden_death_on_invalid_move = sudden_death_on_invalid_move
        self.num_disk_as_reward = num_disk_as_reward
        self.mute = mute
        self.possible_actions_in_obs = possible_actions_in_obs
        self.viewer = None
        n = self.board_size
        self._n, self._W = n, nwords(n)
        self._vec = VecOthelloEnv(1, board_size=n, sudden_death_on_invalid_move=sudden_death_on_invalid_move,
                                  num_disk_as_reward=num_disk_as_reward,
                                  possible_actions_in_obs=possible_actions_in_obs, device=device)
        dev = self._vec.device
        self._planes = 2 if possible_actions_in_obs else 1
        W, nn = self._W, n * n
        # packed staging: boards | legal | meta | reward, done | counts | obs | board_state
        self._o_boards, self._o_legal = 0, 16 * W
        self._o_meta = 24 * W
        self._o_rew = 24 * W + 8
        self._o_done = 24 * W + 12
        self._o_cnt = 24 * W + 16
        self._o_obs = 24 * W + 24
        self._o_abs = self._o_obs + 8 * nn * self._planes
        size = self._o_abs + 8 * nn
        self._stage = torch.zeros(size, dtype=torch.uint8, device=dev)
        self._host = torch.zeros(size, dtype=torch.uint8).pin_memory()
        self._act = torch.zeros(1, dtype=torch.int32, device=dev)
        self._act_host = torch.zeros(1, dtype=torch.int32).pin_memory()
        self._dirty = True
        self._reward = 0
        # Initialize internal states (othello.py:238-242): no possible moves until reset().
        self._vec.set_state(legal=torch.zeros(W, dtype=torch.int64))
        self.action_space = Discrete(n ** 2)
        if possible_actions_in_obs:
            self.observation_space = Box(np.zeros([2, n, n]), np.ones([2, n, n]))
        else:
            self.observation_space = Box(np.zeros([n, n]), np.ones([n, n]))

    # ------------------------------------------------------------ device sync
    def _view(self, off, dtype, count):
        return self._stage[off:off + count * torch.tensor([], dtype=dtype).element_size()].view(dtype)

    def _pull(self):
        """Enqueue state / counts / observations into the staging buffer, one D2H copy, sync."""
        v, lib, s = self._vec, self._vec._lib, self._vec._stream()
        W, n, nn = self._W, self._n, self._n * self._n
        b = self._view(self._o_boards, torch.int64, 2 * W)
        lg = self._view(self._o_legal, torch.int64, W)
        m = self._view(self._o_meta, torch.int16, 1)
        L.check(lib.oth_get_state(v._h, L.ctypes.c_void_p(b.data_ptr()), L.ctypes.c_void_p(m.data_ptr()),
                                  L.ctypes.c_void_p(lg.data_ptr()), s), "oth_get_state")
        c = self._view(self._o_cnt, torch.int32, 2)
        L.check(lib.oth_count_disks(v._h, L.ctypes.c_void_p(c.data_ptr()), s), "oth_count_disks")
        lay = L.OTH_OBS_BOARD_LEGAL if self.possible_actions_in_obs else L.OTH_OBS_BOARD
        o = self._view(self._o_obs, torch.int64, self._planes * nn)
        L.check(lib.oth_observe(v._h, lay, L.OTH_I64, L.ctypes.c_void_p(o.data_ptr()), s), "oth_observe")
        a = self._view(self._o_abs, torch.int64, nn)
        L.check(lib.oth_observe(v._h, L.OTH_OBS_ABSOLUTE, L.OTH_I64, L.ctypes.c_void_p(a.data_ptr()), s),
                "oth_observe")
        self._host.copy_(self._stage, non_blocking=True)
        torch.cuda.current_stream(v.device).synchronize()
        h = self._host.numpy()
        self._boards = h[self._o_boards:self._o_boards + 16 * W].view(np.uint64).copy()
        self._legal = h[self._o_legal:self._o_legal + 8 * W].view(np.uint64).copy()
        meta = int(h[self._o_meta:self._o_meta + 2].view(np.uint16)[0])
        self._reward_dev = int(h[self._o_rew:self._o_rew + 4].view(np.int32)[0])
        self._done_dev = int(h[self._o_done])
        cnt = h[self._o_cnt:self._o_cnt + 8].view(np.int32)
        self._white_cnt, self._black_cnt = np.int64(cnt[0]), np.int64(cnt[1])
        obs = h[self._o_obs:self._o_obs + 8 * nn * self._planes].view(np.int64).copy()
        self._obs = obs.reshape((2, n, n) if self.possible_actions_in_obs else (n, n))
        self._board_state = h[self._o_abs:self._o_abs + 8 * nn].view(np.int64).copy().reshape(n, n)
        self._meta = meta
        self._player_turn = WHITE_DISK if meta & 1 else BLACK_DISK
        self._terminated = bool(meta & 2)
        wc = (meta >> 2) & 3
        self._winner = WHITE_DISK if wc == 1 else (BLACK_DISK if wc == 2 else NO_DISK)
        self._possible_moves = _mask_to_list(self._legal, nn)
        self._dirty = False

    def _sync(self):
        if self._dirty:
            self._pull()

    def _push_meta(self, meta):
        self._vec.set_state(meta=torch.tensor([meta], dtype=torch.int16))
        self._dirty = True

    # ----------------------------------------------- reference attributes
    @property
    def player_turn(self):
        self._sync()
        return self._player_turn

    @player_turn.setter
    def player_turn(self, turn):  # plain attribute write: no recompute (unlike set_player_turn)
        self._sync()
        self._push_meta((self._meta & ~1) | (1 if turn == WHITE_DISK else 0))

    @property
    def terminated(self):
        self._sync()
        return self._terminated

    @terminated.setter
    def terminated(self, value):
        self._sync()
        self._push_meta((self._meta & ~2) | (2 if value else 0))

    @property
    def winner(self):
        self._sync()
        return self._winner

    @winner.setter
    def winner(self, value):
        self._sync()
        code = 1 if value == WHITE_DISK else (2 if value == BLACK_DISK else 0)
        self._push_meta((self._meta & ~12) | (code << 2))

    @property
    def possible_moves(self):
        self._sync()
        return self._possible_moves

    @possible_moves.setter
    def possible_moves(self, moves):
        self._vec.set_state(legal=torch.from_numpy(_list_to_mask(moves, self._n)))
        self._dirty = True

    @property
    def board_state(self):
        self._sync()
        return self._board_state

    @board_state.setter
    def board_state(self, board):
        self._set_absolute(np.asarray(board))

    def _set_absolute(self, board):
        white, black = _board_to_masks(board, self._n)
        self._vec.set_state(boards=torch.from_numpy(np.concatenate([black, white])))
        self._dirty = True

    # ------------------------------------------------------ reference methods
    def reset(self):
        """othello.py:265-271"""
        self._vec.reset()
        self._pull()
        return self.get_observation()

    def step(self, action):
        """othello.py:412-462: returns (observation, reward, done, None)."""
        self._sync()
        if self._terminated:
            raise ValueError('Game has terminated!')
        try:
            a = int(action)
        except (TypeError, ValueError):
            a = -1
        if not -2 ** 31 <= a < 2 ** 31:
            a = -1  # outside int32: not in possible_moves either way
        invalid = a not in self._possible_moves  # only for determine_winner's messages
        self._act_host[0] = a
        self._act.copy_(self._act_host, non_blocking=True)
        rew = self._view(self._o_rew, torch.int32, 1)
        done = self._view(self._o_done, torch.uint8, 1)
        self._vec.step(self._act, rewards=rew, dones=done, observe=False)
        self._pull()
        if self._terminated and not self.mute:
            self._print_result(invalid and self.sudden_death_on_invalid_move)
        return self.get_observation(), self._reward_dev, self._terminated, None

    def _print_result(self, sudden):
        """determine_winner's messages (othello.py:440-441, 476-500); `mute` silences them."""
        if sudden:
            print('sudden death due to rule violation')
        else:
            if self._count_empty() > 0:
                print('No possible moves for either party.')
            print('white: {}, black: {}'.format(self._white_cnt, self._black_cnt))
        print({WHITE_DISK: 'WHITE wins', BLACK_DISK: 'BLACK wins', NO_DISK: 'DRAW'}[self._winner])

    def _count_empty(self):
        return int(self._n ** 2 - self._white_cnt - self._black_cnt)

    def get_possible_actions(self, board=None):
        """othello.py:313-343: ascending legal squares for the mover (or for the
        canonical `board`, mover = +1), recomputed on the device."""
        n = self._n
        if board is None:
            self._sync()
            me = self._player_turn
            board = self._board_state if me == WHITE_DISK else -self._board_state
        mover, opp = _board_to_masks(board, n)
        dev = self._vec.device
        out = legal_moves(n, torch.from_numpy(mover.reshape(1, -1)).to(dev),
                          torch.from_numpy(opp.reshape(1, -1)).to(dev))
        return _mask_to_list(out.cpu().numpy()[0].view(np.uint64), n * n)

    def get_observation(self):
        """othello.py:363-378 (computed by the device observe kernel)."""
        self._sync()
        return self._obs.copy()

    def set_board_state(self, board_state, perspective=WHITE_DISK):
        """othello.py:380-389"""
        state = board_state[0] if np.ndim(board_state) > 2 else board_state
        state = np.array(state)
        self._set_absolute(state if perspective == WHITE_DISK else -state)

    def update_board(self, action):
        """othello.py:391-410 as a standalone call: flip and place for the mover
        without the rest of step() (pass / terminal logic)."""
        self._sync()
        saved = (self._meta, self._legal.copy())
        moves = self._possible_moves
        if action not in moves:
            # the reference flips whatever rays exist even for an illegal square;
            # route through a one-move legal list so the kernel applies them
            self.possible_moves = [action]
        self._vec.step(torch.tensor([int(action)], dtype=torch.int32), observe=False)
        b, _, _ = self._vec.get_state()
        self._vec.set_state(boards=b, meta=torch.tensor([saved[0]], dtype=torch.int16),
                            legal=torch.from_numpy(saved[1].view(np.int64)))
        self._dirty = True

    def set_player_turn(self, turn):
        """othello.py:464-466"""
        self._vec.set_player_turn(turn)
        self._dirty = True

    def count_disks(self):
        """othello.py:468-471: (white_cnt, black_cnt)."""
        self._sync()
        return self._white_cnt, self._black_cnt

    def determine_winner(self, sudden_death=False):
        """othello.py:473-501"""
        self._sync()
        if sudden_death:
            w = BLACK_DISK if self._player_turn == WHITE_DISK else WHITE_DISK
        else:
            w = WHITE_DISK if self._white_cnt > self._black_cnt else (
                BLACK_DISK if self._black_cnt > self._white_cnt else NO_DISK)
        code = 1 if w == WHITE_DISK else (2 if w == BLACK_DISK else 0)
        self._push_meta((self._meta & ~12) | 2 | (code << 2))
        return w

    def print_board(self, print_valid_moves=True):
        """othello.py:345-361"""
        valid_actions = self.get_possible_actions()
        if print_valid_moves:
            board = self.board_state.copy().ravel()
            for p in valid_actions:
                board[p] = 2
            board = board.reshape(*self.board_state.shape)
        else:
            board = self.board_state
        print('Turn: {}'.format('WHITE' if self.player_turn == WHITE_DISK else 'BLACK'))
        print('Valid actions: {}'.format(valid_actions))
        for row in board:
            print(' '.join(map(lambda x: ['B', 'O', 'W', 'V'][x + 1], row)))
        print('-' * 10)

    def render(self, mode='human', close=False):
        if close:
            return
        if mode == 'np_array':
            self.print_board()
        else:
            raise NotImplementedError("the pyglet GUI is out of scope (and broken in the reference: "
                                      "othello.py:5 comments out its renderer)")

    def close(self):
        if self.viewer is not None:
            self.viewer = None

    def seed(self, seed=None):
        return [seed]


class SimpleOthelloEnv(object):
    """SimpleOthelloEnv (othello.py:21-93): random opening plies on top of the base env."""

    metadata = {'render.modes': ['np_array', 'human']}

    def __init__(self, board_size=8, initial_rand_steps=0, seed=0, sudden_death_on_invalid_move=True,
                 render_in_step=False, num_disk_as_reward=False, possible_actions_in_obs=False, device=None):
        self.board_size = board_size
        self.num_disk_as_reward = num_disk_as_reward
        self.env = OthelloBaseEnv(board_size=board_size, num_disk_as_reward=self.num_disk_as_reward,
                                  sudden_death_on_invalid_move=sudden_death_on_invalid_move,
                                  possible_actions_in_obs=possible_actions_in_obs, device=device)
        self.observation_space = self.env.observation_space
        self.action_space = self.env.action_space
        self.render_in_step = render_in_step
        self.initial_rand_steps = initial_rand_steps
        self.rand_seed = seed
        self.rnd = np.random.RandomState(seed=self.rand_seed)
        self.max_rand_steps = 0
        self.rand_step_cnt = 0

    def seed(self, seed=None):
        if seed is not None:
            self.rand_seed = seed
            self.rnd = np.random.RandomState(seed=self.rand_seed)

    def reset(self):
        obs = self.env.reset()
        self.max_rand_steps = self.rnd.randint(low=0, high=self.initial_rand_steps // 2 + 1) * 2
        self.rand_step_cnt = 0
        print('The initial {} steps will be random'.format(self.max_rand_steps))
        return obs

    def step(self, action):
        if self.rand_step_cnt < self.max_rand_steps:
            ix = self.rnd.randint(0, len(self.possible_moves))
            action = self.possible_moves[ix]
            self.rand_step_cnt += 1
        obs, reward, done, _ = self.env.step(action)
        if self.render_in_step:
            self.render()
        return obs, reward, done, None

    def render(self, mode='human', close=False):
        self.env.render(mode=mode, close=close)

    def close(self):
        self.env.close()

    @property
    def player_turn(self):
        return self.env.player_turn

    @property
    def possible_moves(self):
        return self.env.possible_moves


class OthelloEnv(object):
    """OthelloEnv (othello.py:96-214): single-agent view with an embedded opponent policy."""

    metadata = {'render.modes': ['np_array', 'human']}

    def __init__(self, white_policy=None, black_policy=None, protagonist=WHITE_DISK, board_size=8,
                 initial_rand_steps=0, seed=0, sudden_death_on_invalid_move=True, render_in_step=False,
                 num_disk_as_reward=False, possible_actions_in_obs=False, device=None):
        self.board_size = board_size
        self.num_disk_as_reward = num_disk_as_reward
        self.env = OthelloBaseEnv(board_size=board_size, num_disk_as_reward=self.num_disk_as_reward,
                                  sudden_death_on_invalid_move=sudden_death_on_invalid_move,
                                  possible_actions_in_obs=possible_actions_in_obs, device=device)
        self.observation_space = self.env.observation_space
        self.action_space = self.env.action_space
        self.render_in_step = render_in_step
        self.initial_rand_steps = initial_rand_steps
        self.rand_seed = seed
        self.rnd = np.random.RandomState(seed=self.rand_seed)
        self.max_rand_steps = 0
        self.rand_step_cnt = 0
        self.protagonist = protagonist
        if self.protagonist == BLACK_DISK:
            self.opponent = white_policy
        else:
            self.opponent = black_policy

    def switch_color(self):
        self.protagonist = WHITE_DISK if self.protagonist == BLACK_DISK else BLACK_DISK

    def seed(self, seed=None):
        if seed is not None:
            self.rand_seed = seed
            self.rnd = np.random.RandomState(seed=self.rand_seed)
            if self.opponent is not None and hasattr(self.opponent, 'seed'):
                self.opponent.seed(self.rand_seed)

    def reset(self):
        obs = self.env.reset()
        self.max_rand_steps = self.rnd.randint(low=0, high=self.initial_rand_steps // 2 + 1) * 2
        self.rand_step_cnt = 0
        print('The initial {} steps will be random'.format(self.max_rand_steps))
        if hasattr(self.opponent, 'reset'):
            try:
                self.opponent.reset(self)
            except TypeError:
                pass
        if self.env.player_turn == self.protagonist:
            return obs
        action = self.opponent.get_action(obs)
        obs, _, done, _ = self.env.step(action)
        if done:
            print('done==True in reset(), do it again.')
            return self.reset()
        return obs

    def step(self, action):
        assert self.env.player_turn == self.protagonist
        if self.rand_step_cnt < self.max_rand_steps:
            ix = self.rnd.randint(0, len(self.possible_moves))
            action = self.possible_moves[ix]
            self.rand_step_cnt += 1
        obs, reward, done, _ = self.env.step(action)
        if self.render_in_step:
            self.render()
        if done:
            return obs, reward, done, None
        while not done and self.env.player_turn != self.protagonist:
            if self.rand_step_cnt < self.max_rand_steps:
                ix = self.rnd.randint(0, len(self.possible_moves))
                opponent_move = self.possible_moves[ix]
                self.rand_step_cnt += 1
            else:
                opponent_move = self.opponent.get_action(obs)
            obs, reward, done, _ = self.env.step(opponent_move)
            if self.render_in_step:
                self.render()
        return obs, -reward, done, None

    def render(self, mode='human', close=False):
        self.env.render(mode=mode, close=close)

    def close(self):
        self.env.close()

    @property
    def player_turn(self):
        return self.env.player_turn

    @property
    def possible_moves(self):
        return self.env.possible_moves
