"""ORACLE — CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker / CPU baseline.  The product path
(``dl-sound-classification_amd/``) never imports it and fails loudly when the HIP
library is missing.

Pinning: the reference has no tests, fixtures or known-answer vectors.
The restatement is pinned against golden vectors produced by running the reference's
own Python (EnvNetV2 imported as-is; ASTPreprocessor and ASTModel through offline
restatements of torchaudio 2.7.1 / timm 1.0.16) — see ``tests/golden/make_golden.py``.
The third-party layers themselves (torchaudio, timm) are restated from their
published algorithms: parity at that boundary is unpinned by any reference test.
"""
