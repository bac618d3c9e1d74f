"""ORACLE — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import, call, link or execute anything in this directory, and only as the checker
(or as the timed CPU baseline), never as the thing measured or shipped.  The
product package (`distributed-drift-detection_amd/ddm_amd`) never imports it and
fails loudly when its HIP library is missing.

Contents, each citing the reference lines it restates:
  ddm.py         DDM arithmetic (skmultiflow DDM restated, used at DDM_Process.py:133-159)
                 and the per-batch event scan of run_DDM (DDM_Process.py:135-159)
  forest.py      RandomForestClassifier.predict restated on raw tree arrays
                 (DDM_Process.py:110-128 -> sklearn 1.7.2 _forest.py:903-962)
  controller.py  run_DDM_loop restated (DDM_Process.py:170-213): batching, shuffle,
                 lazy refit, refit-on-drift, global MT19937 consumption order
  ddm_scan.c     the same DDM scan in plain C (fast enough for C4-sized parity tests)
  mt_replay.c    the global MT19937 consumption of run_DDM_loop replayed from the seed and
                 the change batches (replay.py: shuffled orders and the final RNG position)

Pinning: tests/golden/ holds outputs of the reference's own function bodies
(DDM_Process.py:94-213, exec'd by tests/golden/make_golden.py) and the tests in
tests/test_oracle.py check this restatement against every one of them.  The DDM
arithmetic itself comes from scikit-multiflow, which is absent from this image:
against upstream skmultiflow it is "parity unpinned" (see DESIGN.md §Oracle).
"""
