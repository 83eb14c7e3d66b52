"""TEST INFRA: an nn.Module wrapper around the CPU oracle (oracle/model_ref.py),
used to drive the host-side training plumbing (training_utils, train_model,
checkpoints, data parallel) on CPU.  Never imported by the package."""
import torch
import torch.nn as nn

from oracle import model_ref


class OracleSeq2Seq(nn.Module):
    def __init__(self, hidden_dim=32, num_heads=2, n_layers=1, seed=0, dropout=0.0):
        super().__init__()
        params = model_ref.seeded_params(model_ref.param_shapes(256, hidden_dim, n_layers, 61), seed)
        self.names = list(params)
        self.plist = nn.ParameterList([nn.Parameter(params[k].clone()) for k in self.names])
        self.num_heads, self.dropout = num_heads, dropout

    def params(self):
        return dict(zip(self.names, self.plist))

    def forward(self, src):
        return model_ref.seq2seq_forward(self.params(), src, self.num_heads, self.dropout, self.training)


class OracleLoss(nn.Module):
    def forward(self, predictions, targets, current_step=None, total_steps=None):
        return model_ref.loss_fn(predictions, targets)
