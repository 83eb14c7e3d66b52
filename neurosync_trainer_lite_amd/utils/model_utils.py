"""Drop-in for the reference ``utils/model_utils.py`` (/root/reference/utils/model_utils.py:9-49)."""
import os

import torch

from .model import Decoder, Encoder, Loss, Seq2Seq
from .optim import FusedAdam


def lr_lambda_for(config):
    """LambdaLR factor, model_utils.py:13-16 (linear decay to 0 over n_epochs)."""
    def lr_lambda(epoch):
        if epoch < config['warmup_epochs']:
            return float(epoch) / float(max(1, config['warmup_epochs']))
        return max(0.0, float(config['n_epochs'] - epoch) / float(max(1, config['n_epochs'] - config['warmup_epochs'])))
    return lr_lambda


def prepare_training_components(config, model):
    """(criterion, optimizer, scheduler) as model_utils.py:9-20.  The optimizer is the
    fused arena Adam (coupled L2, same hyper-parameters and state_dict format as
    torch.optim.Adam).  Like the reference, ``w3`` is not passed to Loss (default 1.0)."""
    criterion = Loss(delta=config['delta'], w1=config['w1'], w2=config['w2'])
    optimizer = FusedAdam(model.parameters(), lr=config['learning_rate'], weight_decay=config['weight_decay'])
    scheduler = torch.optim.lr_scheduler.LambdaLR(optimizer, lr_lambda_for(config))
    return criterion, optimizer, scheduler


def build_model(config, device):
    """model_utils.py:22-26.  On a GPU device the parameter arena is built at once."""
    encoder = Encoder(config['input_dim'], config['hidden_dim'], config['n_layers'], config['num_heads'], config['dropout'])
    decoder = Decoder(config['output_dim'], config['hidden_dim'], config['n_layers'], config['num_heads'], config['dropout'])
    model = Seq2Seq(encoder, decoder, device).to(device)
    model.set_compute_dtype(torch.bfloat16 if config.get('use_amp', True) else torch.float32)
    if config.get('use_fp8', False):  # BASELINE config C5 (not a reference key): fp8 forward projections
        model.set_fp8(True, config.get('fp8_scope', 'attn+enc_ffn1'), config.get('fp8_backward', False))
    if torch.device(device).type == 'cuda':
        model.engine(device)
    return model


def load_model(model_path, config, device):
    """model_utils.py:29-44 (strict load of a reference/own state_dict, eval mode)."""
    model = build_model(config, device)
    state_dict = torch.load(model_path, map_location=device, weights_only=True)
    model.load_state_dict(state_dict, strict=True)
    model.eval()
    return model


def save_final_model(model, final_model_path='out/model.pth'):
    """model_utils.py:46-49."""
    os.makedirs(os.path.dirname(final_model_path), exist_ok=True)
    torch.save(model.state_dict(), final_model_path)
    print(f"Final model saved to {final_model_path}")
