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
import ctypes
import operator

import numpy as np
import torch

from . import _lib as L
from .spaces import Box, Discrete
from .vec_env import VecOthelloEnv, legal_moves, nwords

BLACK_DISK = -1  # othello.py:10-12
NO_DISK = 0
WHITE_DISK = 1


# the set squares of each byte value at each byte offset of a word: possible_moves
# decoded a byte at a time (half the host time of a bit-by-bit loop; config 1 reads
# it on every ply)
_BYTE_SQUARES = [[tuple(8 * k + i for i in range(8) if (b >> i) & 1) for b in range(256)] for k in range(8)]


def _mask_to_list(words, nn):
    out = []
    for wi, w in enumerate(words):
        base = 64 * wi
        for k, b in enumerate((int(w) & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little")):
            if b:
                sq = _BYTE_SQUARES[k][b]
                out.extend(sq if not base else [base + a for a in sq])
    if out and out[-1] >= nn:  # (never for a legal mask: it lies on the board)
        out = [a for a in out if a < nn]
    return out


def _list_to_mask(moves, n):
    W = nwords(n)
    words = [0] * W
    for a in moves:
        a = int(a)
        if 0 <= a < n * n:
            words[a // 64] |= 1 << (a % 64)
    return np.array([w if w < 2 ** 63 else w - 2 ** 64 for w in words], dtype=np.int64)


def _square(action):
    """The square an action names when it is an integer (int, bool, numpy integer,
    0-d integer tensor: anything with __index__), else None."""
    if type(action) is int:
        return action
    try:
        return operator.index(action)
    except TypeError:
        return None


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
        self._planes = 2 if possible_actions_in_obs else 1
        self._layout = L.OTH_OBS_BOARD_LEGAL if possible_actions_in_obs else L.OTH_OBS_BOARD
        self._obs_shape = (2, n, n) if possible_actions_in_obs else (n, n)
        self._sync_fn = self._vec._lib.oth_step_sync
        self._recp = ctypes.c_void_p()
        self._recp_ref = ctypes.byref(self._recp)
        # the record's GreedyPolicy move costs the call about 0.5 us: asked for once a
        # GreedyPolicy reads this env (GreedyPolicy.reset / _greedy_move)
        self._greedy_bit = 0
        self._rec = None  # L.OthRecord over the handle's mapped host record (oth_step_sync)
        self._dirty = True
        # Initialize internal states (othello.py:238-242): no possible moves until reset().
        self._vec.set_state(legal=torch.zeros(self._W, dtype=torch.int64))
        self.action_space = Discrete(n ** 2)
        if possible_actions_in_obs:
            self.observation_space = Box(np.zeros([2, n, n]), np.ones([2, n, n]))
        else:
            self.observation_space = Box(np.zeros([n, n]), np.ones([n, n]))

    # ------------------------------------------------------------ device sync
    def _call(self, step, action=0):
        """oth_step_sync: (step and) record the board in one launch and one wait;
        the record stays in the handle's mapped host buffer, decoded lazily."""
        v = self._vec
        rc = self._sync_fn(v._hv, 0, step | self._greedy_bit, action, self._layout, self._recp_ref, v._stream())
        if rc:
            L.check(rc, "oth_step_sync")
        if self._rec is None or ctypes.addressof(self._rec) != self._recp.value:
            rec = self._rec = L.OthRecord.from_address(self._recp.value)
            nn = self._n * self._n
            self._obs_i8 = np.ctypeslib.as_array(rec.obs)[:self._planes * nn]
            self._abs_i8 = np.ctypeslib.as_array(rec.board_state)[:nn]
            self._legal_u64 = np.ctypeslib.as_array(rec.legal)[:self._W]
        self._dirty = False
        self._moves = None  # decoded possible_moves / board_state of this record
        self._bs = None

    def _pull(self):
        self._call(0)

    def _sync(self):
        if self._dirty:
            self._call(0)

    @property
    def _meta(self):
        self._sync()
        return self._rec.meta

    @property
    def _player_turn(self):
        return WHITE_DISK if self._meta & 1 else BLACK_DISK

    @property
    def _terminated(self):
        return bool(self._meta & 2)

    @property
    def _winner(self):
        wc = (self._meta >> 2) & 3
        return WHITE_DISK if wc == 1 else (BLACK_DISK if wc == 2 else NO_DISK)

    @property
    def _legal(self):
        self._sync()
        return self._legal_u64.copy()

    @property
    def _possible_moves(self):
        self._sync()
        if self._moves is None:
            self._moves = _mask_to_list(self._legal_u64, self._n * self._n)
        return self._moves

    @property
    def _board_state(self):
        self._sync()
        if self._bs is None:
            self._bs = self._abs_i8.astype(np.int64).reshape(self._n, self._n)
        return self._bs

    @property
    def _obs(self):
        self._sync()
        return self._obs_i8.astype(np.int64).reshape(self._obs_shape)

    @property
    def _white_cnt(self):
        self._sync()
        return np.int64(self._rec.white_cnt)

    @property
    def _black_cnt(self):
        self._sync()
        return np.int64(self._rec.black_cnt)

    @property
    def _reward_dev(self):
        return self._rec.reward

    def _greedy_move(self):
        """GreedyPolicy.get_action for the side to move, from the record (-1: no move)."""
        self._sync()
        if self._rec.greedy == L.OTH_RECORD_NO_GREEDY:  # first greedy read: records carry it from now on
            self._greedy_bit = L.OTH_RECORD_GREEDY
            self._call(0)
        return self._rec.greedy

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
        self._call(0)
        return self.get_observation()

    def step(self, action):
        """othello.py:412-462: returns (observation, reward, done, None).  One
        launch steps the board and writes its record to host memory (oth_step_sync).

        Validity is the reference's `action not in self.possible_moves` (:417):
        an integer (int, numpy integer, bool, 0-d integer tensor) is a square; any
        other value is compared with the list by ==, so 19.5 or "19" takes the
        invalid path, while a non-integral member such as 19.0 reaches
        update_board, whose board indexing raises IndexError (:392-406)."""
        if self._terminated:
            raise ValueError('Game has terminated!')
        a = _square(action)
        if a is None:
            if action in self.possible_moves:
                self._index_error(action)
            a = -1
        elif not -2 ** 31 <= a < 2 ** 31:
            a = -1  # outside int32: not in possible_moves either way
        if not self.mute:  # determine_winner's messages need the move's validity
            nn = self._n * self._n
            invalid = not (0 <= a < nn and (int(self._legal_u64[a // 64]) >> (a % 64)) & 1)
        self._call(1, a)
        rec = self._rec
        done = bool(rec.meta & 2)
        if done and not self.mute:
            self._print_result(invalid and self.sudden_death_on_invalid_move)
        return self._obs_i8.astype(np.int64).reshape(self._obs_shape), rec.reward, done, None

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

    def _index_error(self, action):
        """update_board with a value that is no integer (othello.py:391-406): the
        board is negated for a black mover (:395-396), then the first in-board
        neighbour's board[x][y] raises IndexError before any disc is flipped."""
        self._sync()
        if self._player_turn == BLACK_DISK:  # -board_state: the two colours' words swap
            b, _, _ = self._vec.get_state()
            W = self._W
            self._vec.set_state(boards=torch.cat([b[:, W:], b[:, :W]], dim=1))
            self._dirty = True
        raise IndexError("only integers, slices (`:`), ellipsis (`...`), numpy.newaxis (`None`) and integer or "
                         "boolean arrays are valid indices (update_board(%r))" % (action,))

    def update_board(self, action):
        """othello.py:391-410 as a standalone call: for the side to move, flip
        every capped ray from the square and put the mover's disc on it --
        whatever the square held (the reference does not look at it, :407) --
        without the rest of step() (turn, possible_moves and terminal state are
        left as they were).  The flips are the step kernel's, on the board loaded
        live with the square as its one possible move; the square itself is then
        the mover's alone.  A value that is no integer raises IndexError as in
        the reference; so does a square off the board (the reference raises
        there too for action >= N*N, after flipping from the row below the
        board, and wraps negative squares through numpy's negative indexing:
        neither is reachable from step())."""
        a = _square(action)
        if a is None:
            self._index_error(action)
        n = self._n
        if not 0 <= a < n * n:
            raise IndexError("update_board: square %d is off the %dx%d board" % (a, n, n))
        self._sync()
        meta, legal = self._meta, self._legal.copy()
        self._vec.set_state(meta=torch.tensor([meta & ~2], dtype=torch.int16),
                            legal=torch.from_numpy(_list_to_mask([a], n)))
        self._vec.step(torch.tensor([a], dtype=torch.int32), observe=False)
        b, _, _ = self._vec.get_state()
        b = b.cpu().numpy().view(np.uint64).copy()
        other = self._W * ((meta & 1) == 0)  # the opponent's words: white's for a black mover
        b[0, other + a // 64] &= ~np.uint64(1 << (a % 64))
        self._vec.set_state(boards=torch.from_numpy(b.view(np.int64)), meta=torch.tensor([meta], dtype=torch.int16),
                            legal=torch.from_numpy(legal.view(np.int64)))
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
