"""Offline stub of lightning 2.5.2 (absent here): src/datasets/esc50.py imports it only for the
LightningDataModule base class of ESC50DataModule (golden generation instantiates it to run the
reference's own setup(): fold / stratified validation split)."""
