"""Drop-in for utils/csv/save_csv.py:4-62 (LiveLink-style blendshape CSV)."""
import numpy as np
import pandas as pd

BLENDSHAPE_COLUMNS = [
    'EyeBlinkLeft', 'EyeLookDownLeft', 'EyeLookInLeft', 'EyeLookOutLeft', 'EyeLookUpLeft', 'EyeSquintLeft',
    'EyeWideLeft', 'EyeBlinkRight', 'EyeLookDownRight', 'EyeLookInRight', 'EyeLookOutRight', 'EyeLookUpRight',
    'EyeSquintRight', 'EyeWideRight', 'JawForward', 'JawRight', 'JawLeft', 'JawOpen', 'MouthClose', 'MouthFunnel',
    'MouthPucker', 'MouthRight', 'MouthLeft', 'MouthSmileLeft', 'MouthSmileRight', 'MouthFrownLeft',
    'MouthFrownRight', 'MouthDimpleLeft', 'MouthDimpleRight', 'MouthStretchLeft', 'MouthStretchRight',
    'MouthRollLower', 'MouthRollUpper', 'MouthShrugLower', 'MouthShrugUpper', 'MouthPressLeft', 'MouthPressRight',
    'MouthLowerDownLeft', 'MouthLowerDownRight', 'MouthUpperUpLeft', 'MouthUpperUpRight', 'BrowDownLeft',
    'BrowDownRight', 'BrowInnerUp', 'BrowOuterUpLeft', 'BrowOuterUpRight', 'CheekPuff', 'CheekSquintLeft',
    'CheekSquintRight', 'NoseSneerLeft', 'NoseSneerRight', 'TongueOut', 'HeadYaw', 'HeadPitch', 'HeadRoll',
    'LeftEyeYaw', 'LeftEyePitch', 'LeftEyeRoll', 'RightEyeYaw', 'RightEyePitch', 'RightEyeRoll',
]
EMOTION_COLUMNS = ['Angry', 'Disgusted', 'Fearful', 'Happy', 'Neutral', 'Sad', 'Surprised']


def timecode(i, frame_rate=60):
    """HH:MM:SS:FF.mmm of frame i (save_csv.py:39-48 arithmetic)."""
    total_seconds = i * (1 / frame_rate)
    hours, remainder = divmod(total_seconds, 3600)
    minutes, seconds = divmod(remainder, 60)
    milliseconds = (seconds - int(seconds)) * 1000
    frame_number = int(milliseconds / (1000 / frame_rate))
    return f"{int(hours):02}:{int(minutes):02}:{int(seconds):02}:{frame_number:02}.{int(milliseconds):03}"


def save_generated_data_as_csv(generated, output_path, include_emotion_dimensions=False):
    generated = np.array(generated)
    if generated.shape[1] not in [68, 61]:
        raise ValueError(f"Expected generated data to have 68 or 61 columns, but got {generated.shape[1]}")
    if include_emotion_dimensions:
        columns = ['Timecode', 'BlendshapeCount'] + BLENDSHAPE_COLUMNS + EMOTION_COLUMNS
        selected = generated
    else:
        columns = ['Timecode', 'BlendshapeCount'] + BLENDSHAPE_COLUMNS
        selected = generated[:, :61]
    n = generated.shape[0]
    codes = np.array([timecode(i) for i in range(n)]).reshape(-1, 1)
    counts = np.full((n, 1), selected.shape[1])
    # same stacking as the reference: one string array, so values are written
    # with numpy's str() of each float
    data = np.hstack((codes, counts, selected))
    pd.DataFrame(data, columns=columns).to_csv(output_path, index=False)
    print(f"Generated data saved to {output_path}")
