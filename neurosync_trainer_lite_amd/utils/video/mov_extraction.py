"""Drop-in for utils/video/mov_extraction.py:8-62 (clip folder discovery and
ffmpeg audio extraction; host I/O, unchanged behaviour)."""
import os
import subprocess

from ...config import training_config as config


def find_files(folder_path):
    """mov_extraction.py:8-30: last match of each kind wins (os.listdir order)."""
    mov_path = mp4_path = wav_path = facial_csv_path = other_csv_path = None
    audio_features_csv_path = os.path.join(folder_path, 'audio_features.csv')
    for file in os.listdir(folder_path):
        if file.endswith('.mov'):
            mov_path = os.path.join(folder_path, file)
        elif file.endswith('.mp4'):
            mp4_path = os.path.join(folder_path, file)
        elif file.endswith('.wav'):
            wav_path = os.path.join(folder_path, file)
        elif file.endswith('.csv'):
            if 'iPhone_cal' in file:
                facial_csv_path = os.path.join(folder_path, file)
            else:
                other_csv_path = os.path.join(folder_path, file)
    return mov_path, mp4_path, wav_path, facial_csv_path, audio_features_csv_path, other_csv_path


def get_audio(video_path, wav_path, folder_path):
    return extract_audio(video_path, folder_path) if video_path else wav_path


def extract_audio(video_path, output_dir):
    """mov_extraction.py:39-62: mono, config['sr'], cached as audio.wav."""
    audio_path = os.path.join(output_dir, 'audio.wav')
    if os.path.exists(audio_path):
        print(f"Audio already exists at {audio_path}")
        return audio_path
    command = [config['ffmpeg_path'], '-i', video_path, '-ac', '1', '-ar', str(config['sr']), '-y', audio_path]
    try:
        subprocess.run(command, check=True, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        return audio_path
    except (subprocess.CalledProcessError, FileNotFoundError) as e:
        err = e.stderr.decode('utf-8') if isinstance(e, subprocess.CalledProcessError) else str(e)
        print(f"Failed to extract audio from {video_path}: {err}")
        return None
