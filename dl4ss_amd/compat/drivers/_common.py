"""Pieces shared by the py3 driver mirrors: the ground-truth speaker selection, the label-
ordered target assembly, the expanded attention and the two losses, each written as the
reference's training-loop lines do them (cited per function) on the reference-API modules
of ``myNet`` (HIP kernels underneath)."""
import numpy as np
import torch

MSE = torch.nn.MSELoss()


def require_torch_multi_loader_runs(cfg, driver):
    """Fail once, when a driver on the Torch_multi loaders (predata_multiAims_dB / _3dB) starts, if
    ``cfg.AUGMENT_DATA`` is set: those loaders' augmentation line ``signal[s:] + signal[:s]``
    (Torch_multi/predata_multiAims_dB.py:164-166) is a numpy broadcast error for almost every shift,
    so the reference stops at its first source (compat._data.torch_multi_augment restates it) --
    and config_WSJ0_dB.py:112 sets the flag.  Raising here instead of inside the first batch tells
    the user what to change before any model is built."""
    if getattr(cfg, "AUGMENT_DATA", False):
        raise RuntimeError(
            f"{driver}: config_WSJ0_dB.AUGMENT_DATA is True, but the Torch_multi loader this driver uses "
            "cannot augment (predata_multiAims_dB.py:166 raises ValueError on its first source, as in the "
            "reference); set config_WSJ0_dB.AUGMENT_DATA = False to run it.  The TDAA_beta list loaders "
            "(predata_fromList, predata_fromList_cRM_123) do rotate with the flag on.")


def dev():
    return torch.device("cuda")


def cuda(a):
    """``Variable(torch.from_numpy(a)).cuda()``."""
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev())


def ground_truth_selection(train_data, dict_spk2idx, num_labels, multi_label_vector, top_k_mask, alpha=0.5):
    """EvalVer.py:595-605 with config.Ground_truth: the classifier's output is replaced by the
    multi-hot of the batch's speakers, top_k_mask keeps the entries above alpha; returns
    (top_k_mask_mixspeech (B, N_lab) CPU float, top_k_mask_idx list of index arrays, y_map)."""
    y_spk_list = train_data['multi_spk_fea_list']
    y_spk_gtruth, y_map_gtruth = multi_label_vector(y_spk_list, dict_spk2idx)
    mix_speech_output = torch.from_numpy(y_map_gtruth)
    top_k_mask_mixspeech = top_k_mask(mix_speech_output, alpha=alpha, top_k=num_labels)
    top_k_mask_idx = [np.where(line == 1)[0] for line in top_k_mask_mixspeech.numpy()]
    return top_k_mask_mixspeech, top_k_mask_idx, y_map_gtruth


def label_ordered_targets(train_data, top_k_mask_idx, dict_spk2idx, dict_idx2spk, shape):
    """EvalVer.py:632-639 / cRM:730-737: targets stacked in ascending speaker-index order,
    asserting that order is the top-k selection's."""
    y_multi_map = np.zeros(shape, dtype=np.float32)
    for idx, sample in enumerate(train_data['multi_spk_fea_list']):
        y_idx = sorted([dict_spk2idx[spk] for spk in sample.keys()])
        assert y_idx == list(top_k_mask_idx[idx])
        for jdx, oo in enumerate(y_idx):
            y_multi_map[idx, jdx] = sample[dict_idx2spk[oo]]
    return cuda(y_multi_map)


def expanded_attention(att_speech_layer, mix_speech_hidden, queries, B, K, T, F, width):
    """EvalVer.py:615-620: V (B,T,F,E) expanded over the K queries, 'dot' attention per
    (utterance, speaker) -> (B, K, T, F) (cRM: (B, K, T, F, 2))."""
    E = mix_speech_hidden.shape[-1]
    V5 = mix_speech_hidden.view(B, 1, T, F, E).expand(B, K, T, F, E).contiguous()
    att = att_speech_layer(V5.view(-1, T, F, E), queries.reshape(-1, width))
    return att.view(B, K, T, F, 2) if att.dim() == 4 and att.shape[-1] == 2 else att.view(B, K, T, F)


def magnitude_loss(multi_mask, mix_feas, y_multi_map, sum_weight=0.5):
    """EvalVer.py:626-641,658-666: MSE(mask * |X|, Y) + 0.5 MSE(sum_k mask, 1)."""
    B, K, T, F = multi_mask.shape
    predict_multi_map = multi_mask * mix_feas.view(B, 1, T, F).expand(B, K, T, F)
    loss_multi_speech = MSE(predict_multi_map, y_multi_map)
    y_sum_map = torch.ones(B, T, F, device=multi_mask.device)
    predict_sum_map = torch.sum(multi_mask, 1)
    loss_multi_sum_speech = MSE(predict_sum_map, y_sum_map)
    return loss_multi_speech + sum_weight * loss_multi_sum_speech, predict_multi_map, loss_multi_speech, \
        loss_multi_sum_speech
