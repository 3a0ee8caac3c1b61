"""shdpe -- host-side Python binding of the MI355X Shadow path engine.

The product is the C-ABI library ``libshdpe.so`` (include/shd_pathengine.h,
sources in shadow-1_amd/csrc/).  This package only loads it (ctypes), plus the
harness helpers for GraphML input and the synthetic configs.
"""
from .graph import Topology, read_graphml, write_graphml  # noqa: F401
