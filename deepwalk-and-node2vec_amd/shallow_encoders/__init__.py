"""shallow_encoders — MI355X-native DeepWalk / node2vec (skip-gram negative sampling).

Same module layout and public names as the reference package, with the two hot paths
(random-walk generation, SGNS update) running as hand-written gfx950 kernels in
``_lib/libdw_hip.so`` (C ABI: include/dw_hip.h).
"""
__version__ = '0.1.0'
