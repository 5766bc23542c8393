"""OpenAI-compatible request router (the reference's Router component runs the external
``sglang_router`` / ``smg`` image; see ``config/runtimes/srt/*-pd-rt.yaml`` routerConfig).

Policies: ``round_robin``, ``random``, ``power_of_two`` (two random workers, fewer in-flight
wins), ``cache_aware`` (approximate per-worker prefix tree over request text: route to the
worker with the longest cached prefix when the match ratio exceeds ``cache_threshold`` and the
load imbalance is within bounds, else to the least-loaded worker).

Prefill/decode disaggregation (``--pd-disaggregation``): a prefill worker P and a decode
worker D are chosen per request; both receive the request with a shared ``bootstrap_room`` —
P additionally gets D's KV-receiver address — and the client is answered with D's stream
(see :mod:`ome_amd.runtime.disagg`).

Workers come from ``--worker-urls`` / ``--prefill`` / ``--decode`` or from service discovery
(``--service-discovery`` + label selectors) against the manager's REST API (``$OME_API_SERVER``).
"""
from ome_amd.router.policy import CacheAwarePolicy, PowerOfTwoPolicy, RandomPolicy, RoundRobinPolicy, make_policy
from ome_amd.router.server import Router, Worker, build_parser, create_app

__all__ = ["Router", "Worker", "create_app", "build_parser", "make_policy", "RoundRobinPolicy", "RandomPolicy",
           "PowerOfTwoPolicy", "CacheAwarePolicy"]
