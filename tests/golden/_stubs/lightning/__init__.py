"""Offline stub of lightning 2.5.2 (absent here): src/datasets/esc50.py imports it only for the
LightningDataModule base class of ESC50DataModule, which golden generation never instantiates."""
