"""ctypes binding of libdw_hip.so, the C ABI declared in include/dw_hip.h.

This is the only place the host code reaches the HIP kernels. There is no fallback: every
entry point raises ``NativeLibraryError`` when the library is missing, so a device path can
never silently degrade to a CPU implementation.

Device pointers are passed as integers (``tensor.data_ptr()``) and the stream as the integer
``torch.cuda.current_stream().cuda_stream`` handle. ``torch`` is imported before the library is
loaded so that the HIP runtime torch already mapped (soname ``libamdhip64.so.7``) is the one
the library binds to — one runtime, one set of streams.
"""
import ctypes
import os
import threading
from typing import Optional

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_PATH = os.environ.get(   # DW_LIB_PATH: an experimental build (timing studies only)
    'DW_LIB_PATH', os.path.join(os.path.dirname(os.path.abspath(__file__)), '_lib', 'libdw_hip.so'))

DW_OK = 0
DW_E_INVALID_ARG = -1
DW_E_HIP = -2
DW_E_UNSUPPORTED = -3

DW_S_ISOLATED_NODE = 1
DW_S_ZERO_WEIGHT = 2
DW_S_REJECTION_CAP = 4
DW_S_BAD_CSR = 8
DW_S_BAD_INDEX = 16
DW_S_RECORDS_FULL = 32
DW_S_DUP_NEIGHBOR = 64
DW_S_FIXED_RANGE = 128
DW_EXACT_DEFER = 1
DW_EXACT_ADAM = 2

DW_METHOD_DEEPWALK = 0
DW_METHOD_NODE2VEC = 1

ABI_VERSION = 24

_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_f32 = ctypes.c_float
_f64 = ctypes.c_double
_szp = ctypes.POINTER(ctypes.c_size_t)

# name -> (restype, argtypes); mirrors include/dw_hip.h one to one (tests check both ways).
SIGNATURES = {
    'dw_last_error_string': (ctypes.c_char_p, []),
    'dw_abi_version': (ctypes.c_int, []),
    'dw_build_id': (ctypes.c_char_p, []),
    'dw_device_sync': (ctypes.c_int, [_p]),
    'dw_stream_copy': (ctypes.c_int, [_p, _p, _i64, _p]),
    'dw_host_shuffle': (ctypes.c_int, [_p, _p, _i64]),
    'dw_mt_jump_table': (ctypes.c_int, [_i64, _i64, _p, _p, _i64]),
    'dw_mt_uniforms': (ctypes.c_int, [_p, _i32, _i64, _p, _p, _i64, _p, _p, _i64, _p, _i64,
                                      _p]),
    'dw_mt_workspace_words': (ctypes.c_int64, [_i64]),
    'dw_mt_draw': (ctypes.c_int, [_i32, _p, _i32, _i64, _p, _u64, _p, _i64, _p, _p, _i64, _p,
                                  _i64, _p]),
    'dw_csr_validate': (ctypes.c_int, [_p, _p, _i64, _i64, _p, _p]),
    'dw_csr_sort_copy': (ctypes.c_int, [_p, _p, _i64, _i64, _p, _p, _szp, _p]),
    'dw_csr_check_simple': (ctypes.c_int, [_p, _p, _i64, _i64, _p, _p]),
    'dw_adj_hash_offsets': (ctypes.c_int, [_p, _i64, _p, _p, _szp, _p]),
    'dw_adj_hash_build': (ctypes.c_int, [_p, _p, _i64, _p, _i64, _p, _p, _p]),
    'dw_alias_build': (ctypes.c_int, [_p, _p, _i64, _i64, _p, _p, _p, _p, _p, _p]),
    'dw_ingest_workspace_bytes': (ctypes.c_int, [_i32, _i64, _i64, _szp]),
    'dw_rmat_edges': (ctypes.c_int, [_i32, _i64, _p, _p, _u64, _u64, _f64, _f64, _f64, _p, _p, _p,
                                     ctypes.c_size_t, _p]),
    'dw_graph_isolated': (ctypes.c_int, [_p, _i64, _i64, _p, _p, _p, _p, ctypes.c_size_t, _p]),
    'dw_csr_from_edges': (ctypes.c_int, [_p, _i64, _i64, _p, _p, _p, _p, ctypes.c_size_t, _p]),
    'dw_walk_replay': (ctypes.c_int, [_p, _p, _p, _p, _i64, _p, _i64, _i32, _i32, _f64, _f64,
                                      _p, _p, _p, _p]),
    'dw_walk_fast': (ctypes.c_int, [_p, _p, _p, _p, _p, _i64, _p, _i64, _i32, _i32, _f64, _f64,
                                    _u64, _u64, _p, _p, _p]),
    'dw_walk_fast_indexed': (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _p, _i64, _i32,
                                            _i32, _f64, _f64, _u64, _u64, _p, _p, _p]),
    'dw_walk_fast_counted': (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _i64, _p, _i64, _i32, _f64,
                                            _f64, _u64, _u64, _p, _p, _p, _p]),
    'dw_walk_fast_positions': (ctypes.c_int, [_p, _p, _p, _i64, _p, _i64, _i32, _f64, _f64,
                                              _u64, _u64, _p, _p, _p, _p]),
    'dw_edges_inline_build': (ctypes.c_int, [_p, _p, _i64, _i64, _p, _p]),
    'dw_sgns_walks': (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _i64, _i32, _p, _p, _p, _p,
                                     _p, _u64, _u64, _f32, _p, _p, _p, ctypes.c_size_t, _p]),
    'dw_sgns_walks_phase': (ctypes.c_int, [_i32, _p, _i64, _i32, _i32, _i32, _i64, _i32, _p, _p,
                                           _p, _p, _p, _u64, _u64, _f32, _p, _p, _p,
                                           ctypes.c_size_t, _p]),
    'dw_sgns_walks_phase2_piece': (ctypes.c_int, [_i32, _i32, _i64, _p, _i64, _i32, _i32, _i32,
                                                   _i64, _i32, _p, _p, _p, _p, ctypes.c_size_t,
                                                   _p]),
    'dw_sgns_owner_workspace_bytes': (ctypes.c_int, [_i64, _i32, _i32, _i64, _i64, _szp]),
    'dw_sgns_owner_prepare': (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _i64, _i64, _p, _p,
                                             _p, ctypes.c_size_t, _p]),
    'dw_sgns_owner_pass1': (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _i64, _i32, _i32, _i32,
                                           _i64, _i32, _p, _p, _p, _p, _u64, _u64, _f32, _p, _p,
                                           _p, ctypes.c_size_t, _p]),
    'dw_sgns_owner_touch_claim': (ctypes.c_int, [_p, _i64, _i32, _i32, _i64, _p, _i32, _p, _p,
                                                 _p, _p, _i32, _p]),
    'dw_adam_rows': (ctypes.c_int, [_p, _p, _p, _p, _p, _i64, _i32, _p, _p, _i64, _p, _i32, _p,
                                    _i32, _p]),
    'dw_rows_gather': (ctypes.c_int, [_p, _i64, _i32, _p, _p, _i64, _p, _i32, _p]),
    'dw_sgns_owner_pass2': (ctypes.c_int, [_i64, _i32, _i32, _i32, _i64, _i32, _p, _p, _p, _p, _p,
                                           _p, _f32, _f32, _f32, _f32, _f32, _f32, _f32, _p, _p,
                                           ctypes.c_size_t, _p, _p]),
    'dw_sgns_owner_out_catch_up': (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _i64, _i32, _i32,
                                                  _i32, _i64, _p, _u64, _u64, _p, _p, _p, _p, _p,
                                                  _p, _p, _p, _p, _i32, _i32, _p, _p,
                                                  ctypes.c_size_t, _p]),
    'dw_sgns_owner_pass2_lazy': (ctypes.c_int, [_i64, _i32, _i32, _i32, _i64, _i32, _p, _p, _p,
                                                _p, _p, _p, _p, _i32, _i32, _p, _p, _p,
                                                ctypes.c_size_t, _p, _p]),
    'dw_sgns_owner_out_rows': (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _i64, _i32, _i32, _i32,
                                              _i64, _p, _u64, _u64, _f32, _p, _p, _p, _p, _p, _p,
                                              _p, _p, _p, _i32, _p, _p, _p,
                                              ctypes.c_size_t, _p]),
    'dw_sgns_walks_phase2_adam': (ctypes.c_int, [_p, _i64, _i32, _i32, _i32, _i64, _i32, _p, _p,
                                                 _p, _p, _p, _p, _f32, _f32, _f32, _f32, _f32,
                                                 _f32, _f32, _p, _p, ctypes.c_size_t, _p]),
    'dw_sgns_pairs': (ctypes.c_int, [_p, _p, _i64, _i32, _i32, _i64, _i32, _p, _p, _p, _p,
                                     _p, _u64, _u64, _f32, _p, _p, _p, ctypes.c_size_t, _p]),
    'dw_sgns_workspace_bytes': (ctypes.c_int, [_i64, _i32, _i32, _i64, _szp]),
    'dw_sgns_pooled_pairs': (ctypes.c_int, [_p, _i32, _p, _i64, _i32, _i32, _i64, _i32, _p, _p,
                                            _p, _p, _p, _u64, _u64, _f32, _p, _p, _p]),
    'dw_sgns_noise': (ctypes.c_int, [_i64, _i32, _i32, _i64, _u64, _u64, _p, _p]),
    'dw_embedding_renorm_workspace_bytes': (ctypes.c_int, [_i64, _i64, _szp]),
    'dw_embedding_renorm': (ctypes.c_int, [_p, _i64, _i32, _p, _i64, _f64, _p, ctypes.c_size_t,
                                           _p, _p]),
    'dw_pooled_logits': (ctypes.c_int, [_p, _i32, _p, _i64, _i32, _i64, _i32, _p, _p, _i32, _p,
                                        _p, _p]),
    'dw_pooled_logits_backward': (ctypes.c_int, [_p, _i32, _p, _i64, _i32, _i64, _i32, _p, _p,
                                                 _p, _p, _p, _p, _p]),
    'dw_sgns_timing': (ctypes.c_int, [_i32]),
    'dw_sgns_phase_ms': (ctypes.c_int, [ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int64)]),
    'dw_skipgram_logits': (ctypes.c_int, [_p, _p, _i64, _i32, _i64, _i32, _p, _p, _i32, _p, _p,
                                          _p]),
    'dw_skipgram_logits_backward': (ctypes.c_int, [_p, _p, _i64, _i32, _i64, _i32, _p, _p, _p,
                                                   _p, _p, _p, _p]),
    'dw_adam_dense': (ctypes.c_int, [_p, _p, _p, _p, _i64, _f32, _f32, _f32, _f32, _f32, _f32,
                                     _f32, _i32, _p]),
    'dw_adam_dense_to': (ctypes.c_int, [_p, _p, _p, _p, _p, _i64, _f32, _f32, _f32, _f32, _f32,
                                         _f32, _f32, _i32, _i64, _p]),
    'dw_scale': (ctypes.c_int, [_p, _i64, _f32, _p, _p]),
    'dw_step_scalars_bind': (ctypes.c_int, [_p]),
    'dw_step_scalars_bind_at': (ctypes.c_int, [_p, _i64]),
    'dw_step_scalars_advance': (ctypes.c_int, [_p, _p, _i64, _u64, _u64, _p, _p, _i64, _p,
                                               _i64, _p]),
    'dw_step_starts': (ctypes.c_int, [_p, _p, _i64, _p, _i64, _p]),
    'dw_walk_replay_inline': (ctypes.c_int, [_p, _p, _i64, _p, _i64, _i32, _p, _p, _p, _p]),
    'dw_walk_replay_indexed': (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _p, _i64,
                                              _p, _i64, _i32, _f64, _f64, _p, _p, _p, _p, _p]),
    'dw_edge_common_counts': (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p,
                                             _p]),
    'dw_hub_bitmaps': (ctypes.c_int, [_p, _p, _i64, _p, _i64, _i64, _p, _p]),
    'dw_n2v_edge_offsets': (ctypes.c_int, [_p, _p, _p, _i64, _p, _p, _p, _szp, _p]),
    'dw_n2v_edge_index_build': (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _p, _p, _p,
                                               _i64, _i64, _i64, _i64, _i64, _i64, _p, _p, _p,
                                               _p, _szp, _p, _p]),
    'dw_n2v_edge_records': (ctypes.c_int, [_p, _p, _p, _p, _p, _i64, _p, _p]),
    'dw_exact_register': (ctypes.c_int, [_p, _p, _i64, _i32, _i32]),
    'dw_exact_unregister': (ctypes.c_int, [_p]),
    'dw_exact_frac_bits': (ctypes.c_int32, [_f64]),
    'dw_fixed_to_float': (ctypes.c_int, [_p, _p, _i64, _i32, _i32, _p]),
    'dw_walk_replay_positions': (ctypes.c_int, [_p, _p, _p, _i64, _p, _i64, _i32, _f64, _f64,
                                                _p, _p, _p, _p, _p]),
    'dw_adj_hash_positions': (ctypes.c_int, [_p, _p, _i64, _p, _p, _i64, _p, _p, _p]),
    'dw_step_scalars_expand': (ctypes.c_int, [_p, _p, _i64, _p, _i64, _u64, _u64, _p, _p, _i64,
                                              _p, _i64, _p]),
}


class NativeLibraryError(RuntimeError):
    """libdw_hip.so is missing or failed to load (build it with __graft_entry__.build())."""


class DWError(RuntimeError):
    """A libdw_hip entry point returned a negative DW_E_* code."""


_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None


def load() -> ctypes.CDLL:
    """Load (once) and return the library with every signature declared."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f'HIP library not found at {LIB_PATH}; build it with '
                f'`python -c "import __graft_entry__ as g; g.build()"` (hipcc, gfx950)')
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as exc:
            raise NativeLibraryError(f'cannot load {LIB_PATH}: {exc}') from exc
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.dw_abi_version() != ABI_VERSION:
            raise NativeLibraryError(
                f'ABI mismatch: library {lib.dw_abi_version()} != host {ABI_VERSION}; rebuild')
        _lib = lib
        return lib


def call(name: str, *args) -> None:
    """Invoke ``name`` and raise DWError on a negative return code."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != DW_OK:
        msg = lib.dw_last_error_string().decode(errors='replace')
        raise DWError(f'{name} failed ({rc}): {msg}')


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    """Device pointer of a tensor (None -> NULL). Refuses host tensors: no CPU fallback."""
    if t is None:
        return None
    if t.device.type != 'cuda':
        raise ValueError(f'libdw_hip needs device tensors, got a {t.device} tensor')
    if not t.is_contiguous():
        raise ValueError('libdw_hip needs contiguous tensors')
    return t.data_ptr()


def stream(device: Optional[torch.device] = None) -> int:
    """hipStream_t of torch's current stream on ``device``."""
    return torch.cuda.current_stream(device).cuda_stream


def require_device(device) -> torch.device:
    """Resolve the HIP device the hot path runs on; fail loudly without one."""
    if not torch.cuda.is_available():
        raise NativeLibraryError('no HIP device visible: the hot path runs only on MI355X '
                                 '(the CPU restatement lives in oracle/, used by tests only)')
    load()
    dev = torch.device(device) if device is not None else torch.device('cuda',
                                                                       torch.cuda.current_device())
    if dev.type != 'cuda':
        raise ValueError(f'expected a HIP device, got {dev}')
    return dev


def check_status(status: torch.Tensor, what: str) -> None:
    """Synchronising check of a device status word (DW_S_* bits)."""
    s = int(status.item())
    if s == 0:
        return
    if s & DW_S_ISOLATED_NODE:
        raise IndexError(f'{what}: Cannot choose from an empty sequence (walk reached a node '
                         f'without neighbours)')
    if s & DW_S_ZERO_WEIGHT:
        raise ZeroDivisionError(f'{what}: neighbour weights sum to zero')
    if s & DW_S_REJECTION_CAP:
        raise RuntimeError(f'{what}: node2vec rejection sampling exceeded its round cap')
    if s & DW_S_BAD_CSR:
        raise ValueError(f'{what}: malformed CSR graph')
    if s & DW_S_BAD_INDEX:
        raise IndexError(f'{what}: index out of range [0, vocab_size)')
    if s & DW_S_RECORDS_FULL:
        raise RuntimeError(f'{what}: SGNS records exceeded the workspace')
    if s & DW_S_DUP_NEIGHBOR:
        raise ValueError(f'{what}: a CSR row lists the same neighbour twice (the reference\'s '
                         f'networkx.Graph cannot hold a repeated edge)')
    if s & DW_S_FIXED_RANGE:
        raise OverflowError(f'{what}: a gradient term exceeded the deterministic mode\'s '
                            f'fixed-point range (|term| * 2^frac >= 2^51)')
    raise RuntimeError(f'{what}: device status {s:#x}')
