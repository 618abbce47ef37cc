"""See ../__init__.py."""


class LightningDataModule:
    """The slice of lightning 2.5.2's LightningDataModule that ESC50DataModule.__init__ / setup touch:
    save_hyperparameters (a no-op here: nothing is logged)."""

    def __init__(self, *args, **kwargs):
        pass

    def save_hyperparameters(self, *args, **kwargs):
        pass
