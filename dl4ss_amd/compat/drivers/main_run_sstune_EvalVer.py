"""py3 mirror of ``TDAA_beta/main_run_sstune_EvalVer.py`` -- config C2 (BiLSTM-4L magnitude
mask, label-ordered MSE + 0.5 sum-to-one, Adam 2e-4 with the 10-epoch LR halving).

It imports exactly the reference driver's module names (``config_WSJ0_dB as config``,
``predata_fromList``, ``test_multi_labels_speech``, ``bss_test``, ``lrs``, ``librosa``,
``soundfile``; ``compat.install()`` resolves them), defines the driver's module variants
over ``myNet`` (every forward / backward on the HIP kernels) and runs the reference's loop
(``main`` :509-700).  Differences from the reference, each deliberate:

* the training loop runs: the reference's is ``while 0 and True`` (:582, dead code); the
  Discriminator lines (:643-656, :670-671) are not part of the separation step
  and are left out;
* ``torch.optim.Adam`` is the HIP Adam of ``compat.optim`` (same param_groups interface);
* ``config.Load_param`` loads the per-module files through ``dl4ss_amd.checkpoint``-style
  weights_only loads (:545-554) when they exist, and skips them otherwise.

For throughput, ``dl4ss_amd.engine.SepTrainer`` runs the same step fused (bench.py).
"""
import os
import random

import numpy as np
import torch

try:
    from dl4ss_amd import compat as _compat
except ImportError:  # pragma: no cover
    _compat = None
if _compat is not None:
    _compat.install()

import config_WSJ0_dB as config  # noqa: E402
from predata_fromList import prepare_data, prepare_datasize  # noqa: E402,F401
from test_multi_labels_speech import multi_label_vector  # noqa: E402
import bss_test  # noqa: E402,F401
import lrs  # noqa: E402
import librosa  # noqa: E402,F401
import soundfile as sf  # noqa: E402,F401
import myNet  # noqa: E402

from dl4ss_amd.compat.optim import Adam  # noqa: E402
from dl4ss_amd.compat.drivers import _common as C  # noqa: E402
from dl4ss_amd import schedule  # noqa: E402

test_all_outputchannel = 0
test_mode = 1


class MIX_SPEECH(myNet.MIX_SPEECH):
    """EvalVer.py:277-303: nn.LSTM(input_fre, HIDDEN_UNITS, num_layers=4) + Linear + tanh,
    forward returns (V (B,T,F,E), h (B,T,2H))."""

    def __init__(self, input_fre, mix_speech_len):
        super().__init__(input_fre, mix_speech_len, cell="lstm", num_layers=4, return_hidden=True,
                         precision=getattr(config, "PRECISION", "fp32"))


class MIX_SPEECH_classifier(myNet.MIX_SPEECH_classifier):
    """EvalVer.py:305-326: BiLSTM-3L with hidden 2 HIDDEN_UNITS, mean over t, sigmoid."""

    def __init__(self, input_fre, mix_speech_len, num_labels):
        super().__init__(input_fre, mix_speech_len, num_labels, hidden=2 * config.HIDDEN_UNITS, num_layers=3,
                         precision=getattr(config, "PRECISION", "fp32"))


class SPEECH_EMBEDDING(myNet.SPEECH_EMBEDDING):
    """EvalVer.py:348-361 (the gather form, width EMBEDDING_SIZE)."""

    def __init__(self, num_labels, embedding_size, max_num_channel):
        super().__init__(num_labels, embedding_size, max_num_channel, crm=False)


class ADDJUST(myNet.ADDJUST):
    """EvalVer.py:363-377."""

    def __init__(self, hidden_units, embedding_size):
        super().__init__(hidden_units, embedding_size, crm=False)


class ATTENTION(myNet.ATTENTION):
    """EvalVer.py:199-242 ('dot')."""

    def __init__(self, hidden_size, mode='dot'):
        super().__init__(hidden_size, mode, crm=False)


top_k_mask = myNet.top_k_mask


def build(speech_fre, mix_speech_len, num_labels, spk_num_total, lr_data=0.0002):
    """EvalVer.py:522-544 (the Discriminator left out): modules on the GPU + Adam."""
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


def load_params(m, tag="mixdotadjust4lstmdot_WSJ0", epoch=125, classifier="params/param_speech_2mix3lstm_best"):
    """EvalVer.py:545-554 with weights_only loads; missing files are skipped."""
    def ld(mod, path, drop_cnn=False):
        if not os.path.exists(path):
            return False
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if drop_cnn:
            sd = {k: v for k, v in sd.items() if 'cnn' not in k}
        mod.load_state_dict(sd)
        return True

    got = [ld(m['mix_speech_classifier'], classifier, drop_cnn=True)]
    for mod, kind in (('mix_hidden_layer_3d', 'hidden3d'), ('mix_speech_multiEmbedding', 'emblayer'),
                      ('att_speech_layer', 'attlayer'), ('adjust_layer', 'adjlayer')):
        got.append(ld(m[mod], f"params/param_{tag}_{kind}_{epoch}"))
    return got


def train_step(m, optimizer, train_data, dict_spk2idx, dict_idx2spk, num_labels, run_classifier=True):
    """One pass of EvalVer.py:587-641,658-675 on a batch dict.  Returns a dict with the loss
    terms, the masks and the masked prediction (device tensors)."""
    x = C.cuda(train_data['mix_feas'])
    B, T, F = x.shape
    mix_speech_hidden, mix_tmp_hidden = m['mix_hidden_layer_3d'](x)
    if run_classifier:  # :592, computed and then replaced by the ground truth (:598-599)
        with torch.no_grad():
            m['mix_speech_classifier'](x)
    top_k_mask_mixspeech, top_k_mask_idx, _ = C.ground_truth_selection(
        train_data, dict_spk2idx, num_labels, multi_label_vector, top_k_mask)
    mix_speech_multiEmbs = m['mix_speech_multiEmbedding'](top_k_mask_mixspeech, top_k_mask_idx)
    mix_adjust = m['adjust_layer'](mix_tmp_hidden, mix_speech_multiEmbs)
    mix_speech_multiEmbs = mix_adjust + mix_speech_multiEmbs
    assert len(top_k_mask_idx[0]) == len(top_k_mask_idx[-1])
    top_k_num = len(top_k_mask_idx[0])
    multi_mask = C.expanded_attention(m['att_speech_layer'], mix_speech_hidden, mix_speech_multiEmbs, B, top_k_num,
                                      T, F, config.EMBEDDING_SIZE)
    y_multi_map = C.label_ordered_targets(train_data, top_k_mask_idx, dict_spk2idx, dict_idx2spk,
                                          (B, top_k_num, T, F))
    loss, predict_multi_map, l_mask, l_sum = C.magnitude_loss(multi_mask, x, y_multi_map)
    lrs.send('loss mask:', float(l_mask))
    lrs.send('loss sum:', float(l_sum))
    optimizer.zero_grad()
    loss.backward()
    optimizer.step()
    return dict(loss=loss.detach(), loss_mask=l_mask.detach(), loss_sum=l_sum.detach(), mask=multi_mask.detach(),
                pred=predict_multi_map.detach(), top_k_mask_idx=top_k_mask_idx)


def main(max_epoch=None, max_batches=None, log=print):
    """EvalVer.py:509-700 (training); ``max_epoch`` / ``max_batches`` bound a run."""
    np.random.seed(1)
    torch.manual_seed(1)
    random.seed(1)
    spk_global_gen = prepare_data(mode='global', train_or_test='train')
    global_para = next(spk_global_gen)
    spk_all_list, dict_spk2idx, dict_idx2spk, mix_speech_len, speech_fre, total_frames, spk_num_total, \
        batch_total = global_para
    del spk_global_gen
    num_labels = len(spk_all_list)
    m, optimizer = build(speech_fre, mix_speech_len, num_labels, spk_num_total)
    if config.Load_param:
        load_params(m)
    lr_sched = schedule.evalver(optimizer.param_groups[0]['lr'])
    history = []
    for epoch_idx in range(config.MAX_EPOCH if max_epoch is None else max_epoch):
        lr_data = lr_sched.at_epoch_start(epoch_idx)  # :571-575
        for ee in optimizer.param_groups:
            ee['lr'] = lr_data
        lrs.send('lr', lr_data)
        train_data_gen = prepare_data('once', 'train')
        batch_idx = 0
        while True:
            train_data = next(train_data_gen)
            if train_data is False:
                break
            out = train_step(m, optimizer, train_data, dict_spk2idx, dict_idx2spk, num_labels)
            history.append(float(out['loss']))
            log(f"epoch {epoch_idx} batch {batch_idx} loss {history[-1]:.6f} lr {lr_data:g}")
            batch_idx += 1
            if max_batches is not None and batch_idx >= max_batches:
                break
    return m, history


if __name__ == "__main__":
    main()
