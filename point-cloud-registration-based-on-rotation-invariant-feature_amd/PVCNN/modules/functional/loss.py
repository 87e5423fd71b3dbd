"""kl_loss / huber_loss (reference: PVCNN/modules/functional/loss.py:7-17).
Plain torch elementwise losses: no kernel of the path, kept so the
reference's functional namespace is complete."""
import torch
import torch.nn.functional as F

__all__ = ["kl_loss", "huber_loss"]


def kl_loss(x, y):
    p = F.softmax(x.detach(), dim=1)
    return torch.mean(torch.sum(p * (torch.log(p) - F.log_softmax(y, dim=1)), dim=1))


def huber_loss(error, delta):
    a = torch.abs(error)
    q = torch.clamp(a, max=delta)
    return torch.mean(0.5 * q * q + delta * (a - q))
