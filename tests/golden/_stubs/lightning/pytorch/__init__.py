"""See ../__init__.py."""


class LightningDataModule:
    def __init__(self, *args, **kwargs):
        pass
