"""ORACLE -- test infrastructure, NOT product code.

Restatement of the reference's utterance sampling (util/data_loader.py:63-81), used by
tests/test_data.py to pin autoformer_amd.data.Utterances: the same numpy draws in the same
order give the same (uttr, emb) items.
"""
import numpy as np


def reference_item(entry, len_crop):
    """entry = [speaker_id, emb, mel_1, mel_2, ...] with mels already loaded (data_loader.py:46-56).
    Draw the utterance index in [2, len(entry)) (:68); a mel shorter than len_crop is padded at
    the end with zeros (:70-72), a longer one cropped at a uniform offset in [0, T - len_crop)
    (:73-75), an exact one returned as is (:76-77)."""
    pick = np.random.randint(2, len(entry))
    mel = entry[pick]
    n = mel.shape[0]
    if n < len_crop:
        return np.concatenate([mel, np.zeros((len_crop - n, mel.shape[1]), mel.dtype)], axis=0), entry[1]
    if n > len_crop:
        start = np.random.randint(n - len_crop)
        return mel[start:start + len_crop], entry[1]
    return mel, entry[1]
