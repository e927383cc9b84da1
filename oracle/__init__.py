"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's POMCP hot path
(``posggym_baselines/planning/{mcts,node,belief,utils,config}.py``) plus the
build's Driving-v1 generative model and the counter-based RNG that every
random draw on the path is routed through.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import anything from this package, and only as the
checker / reported CPU baseline.  The product path
(``posggym-baselines_amd/``) never imports it.

Pinning: ``oracle.pomcp`` is pinned against the real reference planner,
executed in the build container by ``oracle/ref_harness.py`` (stub-imported,
RNG injected, fake clock for fixed simulation counts).  Its outputs are the
committed fixtures under ``tests/golden/``.  The Driving-v1 dynamics are the
build's own restatement: posggym is not installed and not pinned by the
reference, so parity with posggym's Driving-v1 is UNPINNED.
"""
