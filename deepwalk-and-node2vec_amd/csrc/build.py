"""Build libdw_hip.so (the C-ABI HIP library) in-tree for gfx950.

    python deepwalk-and-node2vec_amd/csrc/build.py [--force] [--jobs N]

Compiles every csrc/*.hip (+ dw_abi.cpp) with hipcc --offload-arch=gfx950 into objects under
csrc/build/, then links shallow_encoders/_lib/libdw_hip.so. Incremental: an object is rebuilt
only when its source or a header is newer. The walk kernels are compiled with
-ffp-contract=off: the replay walker must reproduce CPython's unfused fp64 arithmetic.
"""
import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
OUT_DIR = os.path.join(PKG, 'shallow_encoders', '_lib')
LIB = os.path.join(OUT_DIR, 'libdw_hip.so')
BUILD = os.path.join(HERE, 'build')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('DW_OFFLOAD_ARCH', 'gfx950')

SOURCES = ['dw_abi.cpp', 'dw_host.cpp', 'dw_mt_host.cpp', 'dw_graph.hip', 'dw_walk.hip',
           'dw_sgns.hip', 'dw_adam.hip', 'dw_rmat.hip', 'dw_mt.hip']
# dw_mt_host.cpp is host-only C++ (jump-ahead polynomials over GF(2), carry-less multiplies)
EXTRA = {'dw_walk.hip': ['-ffp-contract=off'], 'dw_mt_host.cpp': ['-x', 'c++']}
HEADERS = [os.path.join(HERE, 'dw_common.h'), os.path.join(REPO, 'include', 'dw_hip.h')]
BASE_FLAGS = ['-x', 'hip', f'--offload-arch={ARCH}', '-O3', '-fPIC', '-std=c++17',
              '-Wall', '-Wno-unused-function', '-I', os.path.join(REPO, 'include')]


def source_id() -> str:
    """SHA-256 (first 16 hex digits) over every source and header the library is built from:
    compiled into libdw_hip.so as dw_build_id(), so a shipped binary can be checked against the
    tree it travels with (tests/test_host.py, __graft_entry__.smoke())."""
    import hashlib
    h = hashlib.sha256()
    for path in [os.path.join(HERE, n) for n in SOURCES] + HEADERS:
        with open(path, 'rb') as f:
            h.update(os.path.basename(path).encode() + b'\0' + f.read())
    return h.hexdigest()[:16]


def _stale(src, obj):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + HEADERS)


def _compile(name, force):
    src = os.path.join(HERE, name)
    obj = os.path.join(BUILD, os.path.splitext(name)[0] + '.o')
    stale = _stale(src, obj)
    if name == 'dw_abi.cpp':   # carries the build id: stale when any source is newer
        stale = stale or not os.path.exists(obj) or any(
            os.path.getmtime(os.path.join(HERE, n)) > os.path.getmtime(obj) for n in SOURCES)
    if not force and not stale:
        return obj, None
    extra = list(EXTRA.get(name, []))
    if name == 'dw_abi.cpp':   # the build id (sources hash): rebuilt whenever any source changes
        extra += [f'-DDW_BUILD_ID="{source_id()}"']
    cmd = [HIPCC] + BASE_FLAGS + extra + ['-c', src, '-o', obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f'{" ".join(cmd)}\n{r.stdout}\n{r.stderr}'
    return obj, None


def build(force: bool = False, jobs: int = 4, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda n: _compile(n, force), SOURCES))
    errors = [e for _, e in results if e]
    if errors:
        raise RuntimeError('hipcc failed:\n' + '\n'.join(errors))
    objs = [o for o, _ in results]
    if force or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB)
                                               for o in objs):
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'link failed:\n{" ".join(cmd)}\n{r.stdout}\n{r.stderr}')
        if verbose:
            print(f'[dw build] linked {LIB}')
    elif verbose:
        print(f'[dw build] up to date: {LIB}')
    return LIB


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('--jobs', type=int, default=4)
    args = ap.parse_args()
    try:
        build(force=args.force, jobs=args.jobs)
    except RuntimeError as exc:
        print(exc, file=sys.stderr)
        sys.exit(1)
