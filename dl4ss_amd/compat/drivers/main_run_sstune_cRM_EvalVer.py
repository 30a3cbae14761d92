"""py3 mirror of ``TDAA_beta/main_run_sstune_cRM_EvalVer.py`` -- config C3 (BiGRU mask net,
complex ratio mask: 10 tanh per query half, inverse compression -1/C log((K-M)/(K+M))
(:688), complex MSE (:720-743), ADDJUST with config.is_SelfTune).

Imports the reference driver's module names (``config_WSJ0_dB``, ``predata_fromList_cRM_123``,
``test_multi_labels_speech``, ``bss_test``, ``librosa``, ``soundfile``) and runs its loop
(:626-753) on the ``myNet`` modules with the HIP Adam.  The inverse compression is
reproduced, not patched: a logit reaching |e| >= 9.02 makes the loss non-finite, as in the
reference.
"""
import random

import numpy as np
import torch

from dl4ss_amd import compat as _compat

_compat.install()

import config_WSJ0_dB as config  # noqa: E402
from predata_fromList_cRM_123 import prepare_data, prepare_datasize  # noqa: E402,F401
from test_multi_labels_speech import multi_label_vector  # noqa: E402
import bss_test  # noqa: E402,F401
import librosa  # noqa: E402,F401
import soundfile as sf  # noqa: E402,F401
import myNet  # noqa: E402

from dl4ss_amd.compat.optim import Adam  # noqa: E402
from dl4ss_amd.compat.drivers import _common as C  # noqa: E402

cRM_k = 10
cRM_C = 0.1


class MIX_SPEECH(myNet.MIX_SPEECH):
    """cRM_EvalVer.py:340-365: nn.GRU(HIDDEN_UNITS, NUM_LAYERS) + Linear + tanh -> (V, h)."""

    def __init__(self, input_fre, mix_speech_len):
        super().__init__(input_fre, mix_speech_len, cell="gru", num_layers=config.NUM_LAYERS, return_hidden=True,
                         precision=getattr(config, "PRECISION", "fp32"))


class MIX_SPEECH_classifier(myNet.MIX_SPEECH_classifier):
    """cRM_EvalVer.py:367-388: BiLSTM(2 HIDDEN_UNITS, NUM_LAYERS)."""

    def __init__(self, input_fre, mix_speech_len, num_labels):
        super().__init__(input_fre, mix_speech_len, num_labels, hidden=2 * config.HIDDEN_UNITS,
                         num_layers=config.NUM_LAYERS, precision=getattr(config, "PRECISION", "fp32"))


class SPEECH_EMBEDDING(myNet.SPEECH_EMBEDDING):
    """cRM_EvalVer.py:390-406: width 2 EMBEDDING_SIZE with is_ComlexMask."""

    def __init__(self, num_labels, embedding_size, max_num_channel):
        super().__init__(num_labels, embedding_size, max_num_channel, crm=bool(config.is_ComlexMask))


class ADDJUST(myNet.ADDJUST):
    def __init__(self, hidden_units, embedding_size):
        super().__init__(hidden_units, embedding_size, crm=bool(config.is_ComlexMask))


class ATTENTION(myNet.ATTENTION):
    def __init__(self, hidden_size, mode='dot'):
        super().__init__(hidden_size, mode, crm=bool(config.is_ComlexMask))


top_k_mask = myNet.top_k_mask


def build(speech_fre, mix_speech_len, num_labels, spk_num_total, lr_data=0.0002):
    """cRM_EvalVer.py:596-613."""
    d = C.dev()
    m = dict(mix_hidden_layer_3d=MIX_SPEECH(speech_fre, mix_speech_len).to(d),
             mix_speech_classifier=MIX_SPEECH_classifier(speech_fre, mix_speech_len, num_labels).to(d),
             mix_speech_multiEmbedding=SPEECH_EMBEDDING(num_labels, config.EMBEDDING_SIZE,
                                                        spk_num_total + config.UNK_SPK_SUPP).to(d),
             att_speech_layer=ATTENTION(config.EMBEDDING_SIZE, 'dot').to(d),
             adjust_layer=ADDJUST(2 * config.HIDDEN_UNITS, config.EMBEDDING_SIZE).to(d))
    optimizer = Adam([{'params': m['mix_hidden_layer_3d'].parameters()},
                      {'params': m['mix_speech_multiEmbedding'].parameters()},
                      {'params': m['mix_speech_classifier'].parameters()},
                      {'params': m['adjust_layer'].parameters()},
                      {'params': m['att_speech_layer'].parameters()}], lr=lr_data)
    return m, optimizer


def train_step(m, optimizer, train_data, dict_spk2idx, dict_idx2spk, num_labels, run_classifier=True):
    """cRM_EvalVer.py:645-752 on one batch dict (complex branch)."""
    x = C.cuda(train_data['mix_feas'])
    B, T, F = x.shape
    W = 2 * config.EMBEDDING_SIZE if config.is_ComlexMask else config.EMBEDDING_SIZE
    mix_speech_hidden, mix_tmp_hidden = m['mix_hidden_layer_3d'](x)
    if run_classifier:
        with torch.no_grad():
            m['mix_speech_classifier'](x)
    top_k_mask_mixspeech, top_k_mask_idx, _ = C.ground_truth_selection(
        train_data, dict_spk2idx, num_labels, multi_label_vector, top_k_mask)
    mix_speech_multiEmbs = m['mix_speech_multiEmbedding'](top_k_mask_mixspeech, top_k_mask_idx)
    if config.is_SelfTune:
        mix_speech_multiEmbs = m['adjust_layer'](mix_tmp_hidden, mix_speech_multiEmbs) + mix_speech_multiEmbs
    top_k_num = len(top_k_mask_idx[0])
    att = C.expanded_attention(m['att_speech_layer'], mix_speech_hidden, mix_speech_multiEmbs, B, top_k_num, T, F, W)
    multi_mask = -1 / cRM_C * torch.log((cRM_k - att) / (cRM_k + att))  # :688
    X = C.cuda(train_data['mix_mag']).view(B, 1, T, F, 2).expand(B, top_k_num, T, F, 2)
    mr, mi = multi_mask[..., 0], multi_mask[..., 1]
    pr = mr * X[..., 0] - mi * X[..., 1]  # :727-728
    pi = mr * X[..., 1] + mi * X[..., 0]
    y = C.label_ordered_targets(train_data, top_k_mask_idx, dict_spk2idx, dict_idx2spk, (B, top_k_num, T, F, 2))
    l_real = C.MSE(pr, y[..., 0])
    l_imag = C.MSE(pi, y[..., 1])
    loss = l_imag + l_real  # :743
    optimizer.zero_grad()
    loss.backward()
    optimizer.step()
    return dict(loss=loss.detach(), loss_real=l_real.detach(), loss_imag=l_imag.detach(), mask=multi_mask.detach(),
                pred=torch.stack([pr, pi], -1).detach())


def main(max_epoch=None, max_batches=None, log=print):
    np.random.seed(1)
    torch.manual_seed(1)
    random.seed(1)
    spk_all_list, dict_spk2idx, dict_idx2spk, mix_speech_len, speech_fre, total_frames, spk_num_total, \
        batch_total = next(prepare_data(mode='global', train_or_test='train'))
    num_labels = len(spk_all_list)
    m, optimizer = build(speech_fre, mix_speech_len, num_labels, spk_num_total)
    history = []
    for epoch_idx in range(config.MAX_EPOCH if max_epoch is None else max_epoch):
        train_data_gen = prepare_data('once', 'train')
        batch_idx = 0
        while True:
            train_data = next(train_data_gen)
            if train_data is False:
                break
            out = train_step(m, optimizer, train_data, dict_spk2idx, dict_idx2spk, num_labels)
            history.append(float(out['loss']))
            log(f"epoch {epoch_idx} batch {batch_idx} loss {history[-1]:.6f}")
            batch_idx += 1
            if max_batches is not None and batch_idx >= max_batches:
                break
    return m, history


if __name__ == "__main__":
    main()
