"""Masked categorical over each board's legal squares, on the GPU.

The learners' policy heads restrict the action distribution to
`possible_moves` one sample at a time in Python:

* ``Policy.act`` (pytorch_a2c_ppo_acktr_gail/a2c_ppo_acktr/model.py:60-99):
  ``FixedCategorical(logits=x[i][possible_moves[i]])``, ``.sample()`` or
  ``.mode()``, ``action = possible_moves[i][idx]``; a board without legal moves
  gets action 0 and log-prob 0 (:69-71);
* ``Policy.evaluate_actions`` (model.py:156-178): log-prob of the stored action
  among the stored choices, 0 when there is none or it is not a choice (:165);
* ``PPO.get_action`` / ``get_test_action`` (ppo.py:228-298): softmax over all
  squares, restricted to ``possible_moves`` and renormalised, then
  ``np.random.choice`` -- the same distribution.

Here one kernel (csrc/masked.hip, C ABI ``oth_masked_sample``) does that for a
whole batch from the (E, W) legal bit masks the engine already holds, so a
rollout step is ``logits = net(obs)`` -> ``masked_sample`` -> ``env.step``
without leaving the device.  The sample is the first legal square whose
cumulative softmax mass exceeds ``u * total`` (``np.random.choice``'s rule)
with ``u`` from the caller or from Philox keyed (seed, env id, counter).
"""
import ctypes

import torch

from . import _lib as L

_MODES = {"sample": L.OTH_MASKED_SAMPLE, "mode": L.OTH_MASKED_MODE}


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _rows(logits, board_size):
    """(n, N*N) or (n, N, N) float32 on a GPU -> a 2-D view with unit column stride."""
    nn = board_size * board_size
    if logits.dtype != torch.float32:
        raise TypeError("logits must be float32, got %s" % logits.dtype)
    if logits.dim() == 3:
        logits = logits.reshape(logits.shape[0], -1)
    if logits.dim() != 2 or logits.shape[1] < nn:
        raise ValueError("logits must be (n, %d) or (n, %d, %d)" % (nn, board_size, board_size))
    if logits.stride(1) != 1:
        logits = logits.contiguous()
    return logits


def _check_legal(legal, n, board_size):
    w = (board_size * board_size + 63) // 64
    if legal.dtype != torch.int64 or tuple(legal.shape) != (n, w):
        raise ValueError("legal must be int64 (%d, %d) bit masks" % (n, w))
    return legal.contiguous()


def masked_sample(logits, legal, board_size, mode="sample", uniforms=None, seed=0, id_base=0, counter=0,
                  log_probs=True, entropy=True, lib=None):
    """Sample (or take the mode of) the masked categorical of every row.

    logits (n, N*N) float32, legal (n, W) int64 bit masks, both on one GPU;
    uniforms: optional (n,) float32 in [0, 1).  Returns (actions int32,
    log_probs float32 or None, entropy float32 or None)."""
    lib = lib if lib is not None else L.load()
    bs = max(4, int(board_size))
    x = _rows(logits, bs)
    n = x.shape[0]
    legal = _check_legal(legal, n, bs)
    if uniforms is not None:
        uniforms = uniforms.to(device=x.device, dtype=torch.float32).contiguous()
    acts = torch.empty(n, dtype=torch.int32, device=x.device)
    lp = torch.empty(n, dtype=torch.float32, device=x.device) if log_probs else None
    ent = torch.empty(n, dtype=torch.float32, device=x.device) if entropy else None
    stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    L.check(lib.oth_masked_sample(bs, n, _ptr(x), x.stride(0), _ptr(legal), _ptr(uniforms), int(seed),
                                  int(id_base), int(counter), _MODES[mode], _ptr(acts), _ptr(lp), _ptr(ent), stream),
            "oth_masked_sample")
    return acts, lp, ent


def masked_log_prob(logits, legal, actions, board_size, entropy=True, full_entropy=False):
    """evaluate_actions: log-prob of `actions` (n,) among each row's legal
    squares (0 where the row has none or the action is not one of them) and
    the entropy per row: of the masked distribution, or with full_entropy=True
    of the unmasked categorical over all squares, which is what
    Policy.evaluate_actions reports (model.py:175, dist.entropy(); it returns
    the mean).  Returns (log_probs float32, entropy float32 or None)."""
    lib = L.load()
    bs = max(4, int(board_size))
    x = _rows(logits, bs)
    n = x.shape[0]
    legal = _check_legal(legal, n, bs)
    acts = actions.to(device=x.device, dtype=torch.int32).reshape(n).contiguous()
    lp = torch.empty(n, dtype=torch.float32, device=x.device)
    ent = torch.empty(n, dtype=torch.float32, device=x.device) if entropy else None
    stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    mode = L.OTH_MASKED_EVAL | (L.OTH_MASKED_FULL_ENTROPY if full_entropy else 0)
    L.check(lib.oth_masked_sample(bs, n, _ptr(x), x.stride(0), _ptr(legal), None, 0, 0, 0, mode,
                                  _ptr(acts), _ptr(lp), _ptr(ent), stream), "oth_masked_sample")
    return lp, ent
