"""Offline restatement of the torchaudio 2.7.1 API surface the reference imports
(uv.lock:2195). Used ONLY by tests/golden/make_golden.py to run the reference's own
preprocessing code in this container; never shipped or imported by the product."""
from . import transforms, functional  # noqa: F401


def load(path):  # pragma: no cover - data files are absent offline
    raise RuntimeError("torchaudio.load is unavailable offline")
