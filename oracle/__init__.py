"""ORACLE — TEST INFRASTRUCTURE ONLY.

A CPU restatement (torch-CPU float32 / numpy float64) of the reference's SVC inference path
(WallaceRao/svc_inference_pipeline). Every function cites the reference file:line it restates.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
package, and only as the checker / the timed CPU baseline. The product package
(`svc_inference_pipeline_amd`) never imports it and has no CPU fallback.

Pinning: tests/golden/*.npz were produced by importing the reference itself in the build container
(tools/make_goldens.py, seeded weights + injected noise) and tests/test_oracle_golden.py checks this
restatement against them. Exceptions, stated in DESIGN.md: Praat's AC pitch (parselmouth absent:
"parity unpinned", known-answer tests on synthetic tones instead).
"""
