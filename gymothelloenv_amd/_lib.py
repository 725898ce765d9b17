"""Loader for the in-tree HIP library liboth_mi355x.so (C ABI: include/othello_mi355x.h).

There is no CPU fallback: if the library is missing or no GPU is visible, the
product classes raise.  `torch` is imported first so that the library's
`libamdhip64.so.7` dependency resolves to the HIP runtime torch already
loaded -- one runtime per process, so torch streams and tensor pointers are
valid arguments.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "liboth_mi355x.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)

OTH_OK = 0
OTH_SUDDEN_DEATH = 1
OTH_DISK_REWARD = 2
OTH_AUTO_RESET = 4
OTH_POLICY_RANDOM = 0
OTH_POLICY_GREEDY = 1
OTH_POLICY_MAXIMIN1 = 2
OTH_POLICY_MAXIMIN2 = 3
OTH_POLICY_MAXIMIN3 = 4
OTH_MAXIMIN_MAX_DEPTH = 10


def OTH_POLICY_MAXIMIN(d):
    return OTH_POLICY_MAXIMIN1 + int(d) - 1
OTH_OBS_BOARD = 0
OTH_OBS_BOARD_LEGAL = 1
OTH_OBS_MAKE_STATE = 2
OTH_OBS_ABSOLUTE = 3
OTH_OBS_LEGAL = 4
OTH_I8, OTH_I32, OTH_I64, OTH_F32, OTH_F64, OTH_BF16 = range(6)
OTH_MASKED_SAMPLE, OTH_MASKED_MODE, OTH_MASKED_EVAL = range(3)
OTH_MASKED_FULL_ENTROPY = 4
OTH_GRAPH_SLOTS = 64
OTH_GRAPH_COUNTER_SHIFT = 40

OTH_RECORD_MAX_WORDS = 4
OTH_RECORD_MAX_SQUARES = 256
OTH_RECORD_GREEDY = 2  # oth_step_sync's `step` bit: the record carries GreedyPolicy's move
OTH_RECORD_NO_GREEDY = -2


class OthRecord(ctypes.Structure):
    """struct oth_record (include/othello_mi355x.h): one board as oth_step_sync
    leaves it in the handle's mapped host buffer."""
    _fields_ = [("black", ctypes.c_uint64 * OTH_RECORD_MAX_WORDS),
                ("white", ctypes.c_uint64 * OTH_RECORD_MAX_WORDS),
                ("legal", ctypes.c_uint64 * OTH_RECORD_MAX_WORDS),
                ("seq", ctypes.c_uint32),
                ("meta", ctypes.c_uint16),
                ("done", ctypes.c_uint8),
                ("planes", ctypes.c_uint8),
                ("reward", ctypes.c_int32),
                ("white_cnt", ctypes.c_int32),
                ("black_cnt", ctypes.c_int32),
                ("greedy", ctypes.c_int32),
                ("obs", ctypes.c_int8 * (2 * OTH_RECORD_MAX_SQUARES)),
                ("board_state", ctypes.c_int8 * OTH_RECORD_MAX_SQUARES)]


# every symbol include/othello_mi355x.h declares: (restype, argtypes)
_P = ctypes.c_void_p
_I32, _U32, _U64, _I64 = ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64
SIGNATURES = {
    "oth_create": (_I32, [_I32, _I32, _U32, _U64, _U32, _I32, _I32, ctypes.POINTER(_P)]),
    "oth_destroy": (_I32, [_P]),
    "oth_reset": (_I32, [_P, _P, _P]),
    "oth_step": (_I32, [_P, _P, _P, _P, _P]),
    "oth_step_observe": (_I32, [_P, _P, _P, _P, _I32, _I32, _P, _P]),
    "oth_step_sync": (_I32, [_P, _I32, _I32, _I32, _I32, ctypes.POINTER(_P), _P]),
    "oth_step_policy": (_I32, [_P, _I32, _I32, _P, _P, _P, _P]),
    "oth_reset_vs": (_I32, [_P, _I32, _P, _P, _P]),
    "oth_step_vs": (_I32, [_P, _I32, _P, _P, _P, _P, _P, _P]),
    "oth_step_vs_observe": (_I32, [_P, _I32, _P, _P, _P, _P, _P, _I32, _I32, _P, _P]),
    "oth_legal": (_I32, [_P, _P, _P]),
    "oth_legal_moves": (_I32, [_I32, _I32, _P, _P, _P, _P]),
    "oth_greedy_actions": (_I32, [_P, _P, _P]),
    "oth_policy_actions": (_I32, [_P, _I32, _P, _P]),
    "oth_observe": (_I32, [_P, _I32, _I32, _P, _P]),
    "oth_get_state": (_I32, [_P, _P, _P, _P, _P]),
    "oth_set_state": (_I32, [_P, _P, _P, _P, _P]),
    "oth_set_player_turn": (_I32, [_P, _I32, _P, _P]),
    "oth_count_disks": (_I32, [_P, _P, _P]),
    "oth_counts": (_I32, [_P, _P, _I32, _P]),
    "oth_counts_vs": (_I32, [_P, _P, _I32, _P]),
    "oth_masked_sample": (_I32, [_I32, _I32, _P, _I64, _P, _P, _U64, _U32, _U64, _I32, _P, _P, _P, _P]),
    "oth_sample_actions": (_I32, [_P, _P, _I64, _P, _U64, _I32, _P, _P, _P, _P]),
    "oth_sample_step": (_I32, [_P, _P, _I64, _P, _U64, _I32, _P, _P, _P, _P, _P, _P]),
    "oth_sample_step_observe": (_I32, [_P, _P, _I64, _P, _U64, _I32, _P, _P, _P, _P, _P, _I32, _I32, _P, _P]),
    "oth_ply_counter": (_U64, [_P]),
    "oth_set_ply_counter": (_I32, [_P, _U64]),
    "oth_graph_begin": (_I32, [_P, _P]),
    "oth_graph_end": (_I32, [_P, _U64, _I32, _P, _P]),
    "oth_graph_offsets": (_I32, [_P, _I32, _P]),
    "oth_graph_release": (_I32, [_P, _I32]),
    "oth_shape": (_I32, [_P, _P, _P, _P]),
    "oth_last_error": (ctypes.c_char_p, []),
    "oth_version": (ctypes.c_char_p, []),
}

_lib = None


class OthelloLibError(RuntimeError):
    pass


def load(require_gpu=True):
    """Load (once) and return the ctypes handle of liboth_mi355x.so.

    require_gpu=False only loads the library (symbol checks on a CPU host)."""
    global _lib
    if _lib is None:
        import torch  # noqa: F401  (HIP runtime first: see module docstring)
        if not os.path.exists(LIB_PATH):
            raise OthelloLibError(
                "%s not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950); there is no CPU fallback" % LIB_PATH)
        from . import build as _build
        have, want = _build.embedded_hash(LIB_PATH), _build.source_hash()
        if have != want:
            raise OthelloLibError(
                "%s was built from other sources (embedded %s, tree %s): rebuild it with "
                "`python -m gymothelloenv_amd.build`" % (LIB_PATH, (have or "none")[:16], want[:16]))
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    if require_gpu:
        import torch
        if not torch.cuda.is_available():
            raise OthelloLibError("no GPU visible: the MI355X Othello engine has no CPU fallback")
    return _lib


def load_path(path):
    """Load another build of the same C ABI (A/B experiments: tools/ab_variants.py)."""
    import torch  # noqa: F401
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)  # an older variant may lack newer entry points
        if fn is not None:
            fn.restype = res
            fn.argtypes = args
    return lib


def check(rc, what="", lib=None):
    if rc != OTH_OK:
        msg = (lib or _lib).oth_last_error().decode() if (lib or _lib) is not None else ""
        raise OthelloLibError("%s failed (%d): %s" % (what or "oth call", rc, msg))
    return rc
