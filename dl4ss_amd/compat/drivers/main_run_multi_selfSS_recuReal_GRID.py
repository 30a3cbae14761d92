"""py3 mirror of ``Torch_multi/main_run_multi_selfSS_recuReal_GRID.py`` -- config C5 (recursive
extraction, inference: the speaker classifier picks the most probable speaker not yet
extracted, its mask is applied, the residual (1 - M) X is fed back, twice; then every
extracted speaker's mask on the original mixture, :383-475).

Imports the reference's names (``config_WSJ0_dB``, ``predata_multiAims_dB``, ``myNet``,
``test_multi_labels_speech``, ``bss_test``) and runs the loop on ``dl4ss_amd.infer.
RecursiveExtractor`` (classifier BiLSTM-3L H = 2 HIDDEN_UNITS + BiGRU mask net, top-k /
speaker choice / residual on the device, one host read per extraction).  The reference
keeps its weights in ``params/`` files; ``load_params`` reads them (weights_only) when they
exist.  Rows of a batch are independent here (the reference runs B = 1).
"""
import random

import numpy as np
import torch

from dl4ss_amd import compat as _compat

_compat.install()

import config_WSJ0_dB as config  # noqa: E402
from predata_multiAims_dB import prepare_data  # noqa: E402
import myNet  # noqa: E402,F401
from test_multi_labels_speech import multi_label_vector  # noqa: E402,F401
import bss_test  # noqa: E402,F401
import librosa  # noqa: E402,F401
import soundfile as sf  # noqa: E402,F401

from dl4ss_amd import checkpoint, engine, infer  # noqa: E402
from dl4ss_amd.compat.drivers import _common as C  # noqa: E402


def build(num_labels=101, B=1, T=None, precision=None):
    """The GRID nets: mask net BiGRU-NUM_LAYERS (no ADDJUST) + classifier BiLSTM-3L H = 2 HIDDEN_UNITS."""
    prec = precision or getattr(config, "PRECISION", "fp32")
    T = T or (1 + config.MAX_LEN // config.FRAME_SHIFT)
    net = engine.SepNet(cell="gru", num_layers=config.NUM_LAYERS, hidden=config.HIDDEN_UNITS,
                        emb=config.EMBEDDING_SIZE, num_labels=num_labels, adjust=False, device="cuda")
    cnet = infer.ClassifierNet(hidden=2 * config.HIDDEN_UNITS, num_layers=3, num_labels=num_labels, device="cuda")
    ext = infer.RecursiveExtractor(net, cnet, B, T, precision=prec, alpha=-0.3, top_k=3, max_steps=2)
    return net, cnet, ext


def load_params(net, cnet, hidden3d=None, emblayer=None, classifier=None):
    import os

    files = {k: v for k, v in (("hidden3d", hidden3d), ("emblayer", emblayer)) if v and os.path.exists(v)}
    if files:
        checkpoint.load_reference_params(net, **files)
    if classifier and os.path.exists(classifier):
        checkpoint.load_reference_classifier(cnet, classifier)


def extract(ext, train_data, dict_idx2spk):
    """One batch: the speakers extracted in order (names), their masks on the original
    mixture (B, 2, T, F) and the masked predictions (B, 2, T, F)."""
    X = torch.from_numpy(np.ascontiguousarray(train_data['mix_feas'])).cuda()
    out = ext.run(X)
    spk = out['spk'].cpu().numpy()
    names = [[dict_idx2spk.get(int(s)) if s >= 0 else None for s in row] for row in spk]
    pred = out['masks'] * X[:, None]
    return names, out['masks'], pred


def main(max_batches=2, log=print):
    C.require_torch_multi_loader_runs(config, "main_run_multi_selfSS_recuReal_GRID")
    np.random.seed(1)
    torch.manual_seed(1)
    random.seed(1)
    spk_all_list, dict_spk2idx, dict_idx2spk, mix_speech_len, speech_fre, total_frames, spk_num_total = \
        next(prepare_data(mode='global', train_or_test='train'))
    net, cnet, ext = build(len(spk_all_list), B=config.BATCH_SIZE, T=mix_speech_len)
    results = []
    for batch_idx in range(max_batches):
        train_data = next(prepare_data('once', 'eval_test'))
        names, masks, pred = extract(ext, train_data, dict_idx2spk)
        results.append(names)
        log(f"batch {batch_idx}: extracted {names}")
    return results


if __name__ == "__main__":
    main()
