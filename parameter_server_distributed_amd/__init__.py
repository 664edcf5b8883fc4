"""MI355X-native parameter-server training runtime.

Roles (same as the reference araju6/parameter-server-distributed): a coordinator (worker registry,
heartbeats, PS address / shard map), parameter-server shards (parameters + optimizer state + the
fused update) and workers (pull -> forward/backward -> push). The control plane speaks the
reference's gRPC services; the tensor data plane is RCCL over xGMI (push = reduce-scatter,
pull = all-gather) with the PS shards held in HBM and updated by hand-written gfx950 kernels.

Sub-packages:
  ops/       Python entry points for the HIP kernels (fused optimizer, reduce, pack/cast, fp8, GEMM)
  models/    MLP, ResNet-50, BERT-base, Wide-ResNet-101 (random init, synthetic data)
  parallel/  data plane: flat bucketed shards, RCCL/gloo transports, sync + bounded-staleness async
  runtime/   coordinator / parameter-server / worker role logic
  rpc/       gRPC wire schema (coordinator.proto / parameter_server.proto) and service glue
  cli/       argv-compatible entry points (coordinator, parameter_server, worker_main)
  utils/     logging, metrics, tracing, config
"""
from __future__ import annotations

import importlib
import os

__version__ = "0.1.0"

_NATIVE = None


def native():
    """Return the compiled extension ``_C`` (HIP kernels + C++ cores).

    Fails loudly: there is no silent pure-PyTorch fallback for the kernels on a GPU box. Set
    ``PSD_AUTOBUILD=1`` to build it on first use (the driver calls ``__graft_entry__.build()``).
    """
    global _NATIVE
    if _NATIVE is None:
        import torch  # noqa: F401  (torch's HIP runtime must be loaded before _C)

        try:
            _NATIVE = importlib.import_module(__name__ + "._C")
        except ImportError as e:
            if os.environ.get("PSD_AUTOBUILD", "0") == "1":
                from . import _build

                _build.build()
                _NATIVE = importlib.import_module(__name__ + "._C")
            else:
                raise ImportError(
                    "parameter_server_distributed_amd._C is not built; run "
                    "`python -m parameter_server_distributed_amd._build` (or __graft_entry__.build())"
                ) from e
    return _NATIVE
