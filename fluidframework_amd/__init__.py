"""fluidframework_amd — MI355X-native batched replay engine for Fluid's merge-tree sequence CRDT.

The hot path (sequenced-op replay + SnapshotV1 emission for many SharedString documents) runs as
HIP kernels on gfx950 behind the C ABI in include/mte.h; `mte` is the Python mirror of that ABI.
"""
from .mte import Builder, Engine, MergeTreeClient, MteError, lib  # noqa: F401
