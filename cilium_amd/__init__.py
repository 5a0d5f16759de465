"""cilium_amd — MI355X-native batch packet-verdict engine for Cilium's L3/L4 datapath.

The product is the C-ABI library ``cilium_amd/_lib/libcilium_hip.so`` (HIP kernels for
gfx950 + the map store); this package holds its sources (``csrc/``), a thin ctypes
binding of the C-ABI (``lib``), the synthetic BASELINE workloads (``synth``), the
address-pair sharding of conntrack over GPUs (``shard``) and the build (``build``).
Importing the package does not load the library; ``cilium_amd.lib.load()`` does and
raises if it is missing.
"""
__version__ = "0.1.0"
