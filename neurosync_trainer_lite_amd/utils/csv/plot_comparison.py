"""Drop-in for utils/csv/plot_comparison.py (JawOpen ground truth vs generated)."""
import numpy as np
import pandas as pd


def pad_data(df1, df2):
    max_len = max(len(df1), len(df2))
    if len(df1) < max_len:
        df1 = pd.concat([df1, pd.DataFrame(0, index=np.arange(max_len - len(df1)), columns=df1.columns)],
                        ignore_index=True)
    elif len(df2) < max_len:
        df2 = pd.concat([df2, pd.DataFrame(0, index=np.arange(max_len - len(df2)), columns=df2.columns)],
                        ignore_index=True)
    return df1, df2


def plot_comparison(ground_truth_path, generated_path, output_image_path):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    ground_truth, generated = pad_data(pd.read_csv(ground_truth_path), pd.read_csv(generated_path))
    ground_truth, generated = ground_truth.head(512), generated.head(512)
    timecodes = ground_truth['Timecode'].astype(str)
    plt.figure(figsize=(20, 20))
    for feature in ['JawOpen']:
        plt.plot(timecodes, ground_truth[feature], label=f'Ground Truth {feature}')
        plt.plot(timecodes, generated[feature], label=f'Generated {feature}', linestyle='dashed')
    plt.legend()
    plt.xticks(rotation=45)
    plt.xlabel('Timecode')
    plt.ylabel('Feature Value')
    plt.title('Comparison of Ground Truth and Generated Facial Features')
    plt.tight_layout()
    plt.savefig(output_image_path, dpi=100)
    plt.close()
    print(f"Comparison plot saved to {output_image_path}")
