"""Drop-in for utils/validation.py:14-137 (per-epoch validation clip: features
on the GPU, batched chunk inference, CSV + plot + comparison statistics).

The reference writes the CSV and the plot from child processes
(multiprocessing.Process under ``lock``); here they are written in-process,
under the same lock, because forking a process that holds a GPU context is
not safe on ROCm.  The JawOpen comparison plot (utils/csv/plot_comparison.py)
is cosmetic and out of scope; the statistics it sits
beside are written."""
import os

import numpy as np
import pandas as pd

from ..config import training_config
from .audio.extraction.extract_features import extract_audio_features
from .audio.processing.audio_processing import process_audio_features
from .csv.save_csv import BLENDSHAPE_COLUMNS, save_generated_data_as_csv

DIMENSION_LABELS = BLENDSHAPE_COLUMNS


def generate_and_save_facial_data(epoch, audio_path, model, ground_truth_path, lock, device):
    audio_features, _ = extract_audio_features(audio_path)
    generated_facial_data = process_audio_features(audio_features, model, device, training_config)
    base_dir = "dataset/validation_plots"
    stats_dir = os.path.join(base_dir, "stats")
    os.makedirs(base_dir, exist_ok=True)
    os.makedirs(stats_dir, exist_ok=True)
    output_csv_path = os.path.join(base_dir, f"generated_facial_data_epoch_{epoch + 1}.csv")
    with lock:
        save_generated_data_as_csv(generated_facial_data, output_csv_path)
    output_stats_path = os.path.join(stats_dir, f"comparison_stats_epoch_{epoch + 1}.txt")
    return save_comparison_stats(output_csv_path, ground_truth_path, output_stats_path)


def comparison_stats(generated, ground_truth):
    """validation.py:75-124 on aligned arrays -> (overall, per-dimension)."""
    n = min(generated.shape[0], ground_truth.shape[0])
    generated, ground_truth = generated[:n], ground_truth[:n]
    diff = ground_truth - generated
    abs_diff = np.abs(diff)
    pct = np.divide(abs_diff, np.abs(ground_truth), out=np.zeros_like(abs_diff), where=np.abs(ground_truth) > 1e-6) * 100
    pct = np.nan_to_num(pct, nan=0.0, posinf=0.0, neginf=0.0)
    overall = {
        'Mean Absolute Error (MAE)': np.nanmean(abs_diff),
        'Mean Absolute Percentage Error (MAPE)': np.nanmean(pct),
        'Mean Squared Error (MSE)': np.nanmean(diff ** 2),
        'Root Mean Squared Error (RMSE)': np.sqrt(np.nanmean(diff ** 2)),
        'Correlation Coefficient (r)': (np.corrcoef(generated.flatten(), ground_truth.flatten())[0, 1]
                                        if np.nanstd(generated) > 1e-6 and np.nanstd(ground_truth) > 1e-6
                                        else float('nan')),
    }
    per_dim = {}
    for i, label in enumerate(DIMENSION_LABELS):
        if np.nanstd(ground_truth[:, i]) > 1e-6 and np.nanstd(generated[:, i]) > 1e-6:
            r = np.corrcoef(generated[:, i], ground_truth[:, i])[0, 1]
        else:
            r = float('nan')
        per_dim[label] = {
            'MAE': np.nanmean(abs_diff[:, i]),
            'MAPE': np.nanmean(pct[:, i]),
            'MSE': np.nanmean(diff[:, i] ** 2),
            'RMSE': np.sqrt(np.nanmean(diff[:, i] ** 2)),
            'Correlation Coefficient': r,
        }
    return overall, per_dim


def save_comparison_stats(generated_data_path, ground_truth_path, output_stats_path):
    generated = pd.read_csv(generated_data_path).iloc[:, 2:2 + len(DIMENSION_LABELS)].values.astype(np.float64)
    ground_truth = pd.read_csv(ground_truth_path).iloc[:, 2:].values.astype(np.float64)
    overall, per_dim = comparison_stats(generated, ground_truth)
    with open(output_stats_path, 'w') as f:
        f.write("Overall Comparison Statistics:\n")
        for k, v in overall.items():
            f.write(f"{k}: {v:.4f}\n")
        f.write("\nPer-Dimension Statistics:\n")
        for label, stats in per_dim.items():
            f.write(f"{label}:\n")
            for k, v in stats.items():
                f.write(f"  {k}: {v:.4f}\n")
    print(f"Comparison statistics saved to {output_stats_path}")
    return overall
