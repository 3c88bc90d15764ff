"""CPU restatement of the reference's co-teaching loss (TEST INFRASTRUCTURE:
only tests/ may import it; the product path is ngnn.losses.CTLoss on the
device).

Follows ``CTLoss.forward`` of src/utils/losses.py:19-49 step by step:
per-row cross entropy of both models (:20, :24), ascending argsort of each
(:21, :25 -- np.argsort's default quicksort leaves the order of tied losses
unspecified; this restatement breaks ties by row index, a stable sort, which
the device kernel follows too), num_remember = int((1 - forget_rate) * B)
(:29-30), pure ratios over ``noise_or_not[ind[kept]]`` (:32-33), and the
exchange: model 1 is trained on the rows model 2 kept and vice versa
(:43-45).  Pinned against the reference's own CTLoss run on the same inputs
(tests/golden/ct_loss_*.npz, made by tests/golden/make_golden.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def ct_loss(y_1, y_2, y_noise, forget_rate, ind, noise_or_not):
    loss_1 = F.cross_entropy(y_1, y_noise, reduction="none")
    ind_1_sorted = torch.sort(loss_1.detach(), stable=True).indices
    loss_2 = F.cross_entropy(y_2, y_noise, reduction="none")
    ind_2_sorted = torch.sort(loss_2.detach(), stable=True).indices
    remember_rate = 1 - forget_rate
    num_remember = int(remember_rate * len(loss_1))
    pure_ratio_1 = torch.sum(noise_or_not[ind[ind_1_sorted[:num_remember]]]) / float(num_remember)
    pure_ratio_2 = torch.sum(noise_or_not[ind[ind_2_sorted[:num_remember]]]) / float(num_remember)
    ind_1_update = ind_1_sorted[:num_remember]
    ind_2_update = ind_2_sorted[:num_remember]
    ind_noisy_1 = ind_1_sorted[num_remember:]
    ind_noisy_2 = ind_2_sorted[num_remember:]
    loss_1_update = F.cross_entropy(y_1[ind_2_update], y_noise[ind_2_update])
    loss_2_update = F.cross_entropy(y_2[ind_1_update], y_noise[ind_1_update])
    return (loss_1_update, loss_2_update, pure_ratio_1, pure_ratio_2, ind_1_update, ind_2_update,
            ind_noisy_1, ind_noisy_2)
