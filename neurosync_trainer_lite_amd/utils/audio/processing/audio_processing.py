"""Drop-in for utils/audio/processing/audio_processing.py:1-140 (clip inference).

Same chunking (frame_size frames, ``overlap`` frames shared between chunks),
reflect padding of a short chunk, linear cross-fade of the overlap, tail chunk,
and /100 rescale.  Chunks do not depend on each other, so all of them go through
the model in a few batched forwards (the reference runs one forward per chunk,
:63-83); blending stays sequential on the host exactly as the reference does it.
"""
import numpy as np
import torch

MAX_CHUNKS_PER_FORWARD = 256


def concatenate_outputs(all_decoded_outputs, num_frames):
    return np.concatenate(all_decoded_outputs, axis=0)[:num_frames]


def ensure_2d(final_decoded_outputs):
    if final_decoded_outputs.ndim == 3:
        final_decoded_outputs = final_decoded_outputs.reshape(-1, final_decoded_outputs.shape[-1])
    return final_decoded_outputs


def pad_audio_chunk(audio_chunk, frame_length, num_features):
    """audio_processing.py:14-23 (numpy 'reflect' pad, then the tail of it)."""
    if audio_chunk.shape[0] < frame_length:
        pad_length = frame_length - audio_chunk.shape[0]
        padding = np.pad(audio_chunk, pad_width=((0, pad_length), (0, 0)), mode='reflect')
        audio_chunk = np.vstack((audio_chunk, padding[-pad_length:, :num_features]))
    return audio_chunk


def decode_audio_chunk(audio_chunk, model, device):
    """audio_processing.py:25-31 (one chunk; kept for API compatibility)."""
    return _decode_batch([audio_chunk], model, device)[0]


def _decode_batch(chunks, model, device):
    outs = []
    with torch.no_grad():
        for i in range(0, len(chunks), MAX_CHUNKS_PER_FORWARD):
            src = torch.as_tensor(np.stack(chunks[i:i + MAX_CHUNKS_PER_FORWARD]), dtype=torch.float32).to(device)
            enc = model.encoder(src)
            outs.extend(model.decoder(enc).cpu().numpy())
    return outs


def blend_chunks(chunk1, chunk2, overlap):
    """audio_processing.py:33-48."""
    actual_overlap = min(overlap, len(chunk1), len(chunk2))
    if actual_overlap == 0:
        return np.vstack((chunk1, chunk2))
    blended = np.copy(chunk1)
    # per-row Python-float weights applied in the arrays' own precision, as the
    # reference's scalar loop does (bit-identical)
    dt = np.result_type(chunk1, chunk2)
    a = [i / actual_overlap for i in range(actual_overlap)]
    alpha = np.array(a, dtype=dt)[:, None]
    keep = np.array([1 - x for x in a], dtype=dt)[:, None]
    blended[-actual_overlap:] = keep * chunk1[-actual_overlap:] + alpha * chunk2[:actual_overlap]
    return np.vstack((blended, chunk2[actual_overlap:]))


def chunk_plan(num_frames, frame_length, overlap):
    """Chunk start/end indices of the reference's while loop (:62-83)."""
    plan, start = [], 0
    while start < num_frames:
        plan.append((start, min(start + frame_length, num_frames)))
        start += frame_length - overlap
    return plan


def process_audio_features(audio_features, model, device, config):
    """audio_processing.py:50-112 -> [num_frames, 61] (blendshapes / 100)."""
    frame_length = config['frame_size']
    overlap = config.get('overlap', 16)
    num_features = audio_features.shape[1]
    num_frames = audio_features.shape[0]
    model.eval()
    plan = chunk_plan(num_frames, frame_length, overlap)
    chunks = [pad_audio_chunk(audio_features[s:e], frame_length, num_features) for s, e in plan]
    decoded = _decode_batch(chunks, model, device)
    all_decoded_outputs = []
    for (s, e), out in zip(plan, decoded):
        out = out[:e - s]
        if all_decoded_outputs:
            all_decoded_outputs.append(blend_chunks(all_decoded_outputs.pop(), out, overlap))
        else:
            all_decoded_outputs.append(out)
    current_length = sum(len(c) for c in all_decoded_outputs)
    if current_length < num_frames:
        remaining = num_frames - current_length
        chunk = pad_audio_chunk(audio_features[num_frames - remaining:num_frames], frame_length, num_features)
        all_decoded_outputs.append(_decode_batch([chunk], model, device)[0][:remaining])
    final = ensure_2d(np.concatenate(all_decoded_outputs, axis=0)[:num_frames])
    final[:, :61] /= 100
    return final


def zero_columns(data):
    columns_to_zero = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60]
    out = np.copy(data)
    out[:, columns_to_zero] = 0
    return out
