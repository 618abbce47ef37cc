"""Placeholder: the out-of-scope CNN preprocessor's torchvision transforms."""


def __getattr__(name):
    class _Placeholder:
        def __init__(self, *a, **k):
            raise RuntimeError(f"torchvision.transforms.{name} is not available offline")
    return _Placeholder
