"""CPU oracle for the NeuroSync Trainer Lite training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``neurosync_trainer_lite_amd/`` imports
this package; only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may use it, and only as the checker (or
the timed CPU baseline), never as a compute path of the product.

Every function restates the reference algorithm (``/root/reference``) and cites
the file:line it follows.  Parity pinning: see ``oracle/README.md``.
"""
