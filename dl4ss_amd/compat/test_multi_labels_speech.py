"""``multi_label_vector`` of Torch_multi/test_multi_labels_speech.py:285-298 (the rest of
that file trains the speaker classifier and is out of scope)."""
import numpy as np


def multi_label_vector(x, dict_name2idx):
    """x: list of per-sample dicts keyed by speaker name -> (y_spk: list of index lists in
    the dicts' key order, y_map: (B, N_lab) float32 multi-hot)."""
    y_spk, y_aim = [], []
    length = len(dict_name2idx)
    for sample in x:
        vec = [0] * length
        line = [dict_name2idx[spk] for spk in sample.keys()]
        for l in line:
            vec[l] = 1
        y_spk.append(line)
        y_aim.append(vec)
    return y_spk, np.array(y_aim, dtype=np.float32)
