"""Multi-GPU layer: one rank per MI355X, sessions sharded over one SO_REUSEPORT port (DP),
optional backend-stream placement across ranks with an RCCL all-gather exchange (EP).

* :mod:`.topology` — rank environment, KFD xGMI link discovery
* :mod:`.exchange` — exchange transport / rendezvous settings shared by every rank
* :mod:`.launcher` — ``qmx serve --gpus N`` node launcher
The collective itself is native (``csrc/qmx_exchange.cpp``).
"""
from .exchange import cluster_config, exchange_env  # noqa: F401
from .topology import RankEnv, gpu_links, summary  # noqa: F401
