"""Inputs of tests/golden/golden_aug.npz, regenerated from oracle/synth.py (splitmix64 counters) on
whichever machine runs the tests; make_golden.py fed the same arrays to the reference."""
import numpy as np

from oracle.synth import hash_uniform, synth_waveform

AUG_BC_SCALES = (1.0, 0.05, 0.5, 1.0, 0.02, 0.8)
AUG_BC_LABELS = (0, 0, 1, 2, 2, 3)
AUG_MIX_LABELS = (5, 9, 5, 2)
AUG_STRETCH_CFG = {"time_stretch": [0.8, 1.25], "gain_shift": [-6, 6]}
AUG_SPEC_CASES = [((1, 128, 1379), 192, 48)] * 4 + [((1, 16, 40), 8, 2)] * 2 + [((1, 16, 6), 8, 2)]


def aug_bc_pool():
    return [synth_waveform(700 + i, 1, 22_050) * np.float32(s) for i, s in enumerate(AUG_BC_SCALES)]


def aug_mix_pool():
    return [hash_uniform(760 + i, (1, 128, 1379)) for i in range(len(AUG_MIX_LABELS))]


def aug_spec_input(s):
    shape = AUG_SPEC_CASES[s][0]
    return hash_uniform(51 + s, shape)


def aug_stretch_input():
    return synth_waveform(790, 1, 22_050)


def aug_crop_clip(i):
    return synth_waveform(800 + i, 1, 44_100)
