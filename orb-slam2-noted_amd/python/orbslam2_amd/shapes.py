"""Launch shapes the benchmark measures, shared by bench.py and the GPU parity tests so the tested
shape and the measured shape cannot diverge.

C2: a 512-frame stereo stream at 1241x376, 384 pairs per step over 3 pipeline
engines. C3: batches of 256 TUM RGB-D frames alternating over 4 engines.
"""
C2_W, C2_H = 1241, 376
C2_STREAM_FRAMES = 512   # "A stream of 512 frames" (left seed 2 + t)
C2_BATCH = 384           # stereo pairs per step (= per orbx_pipeline_stereo_batch call)
C2_ENGINES = 3           # orbx_pipeline engines the batch is split over

C3_BATCH = 256           # RGB-D frames per batch
C3_ENGINES = 4           # engines consecutive batches alternate over


def c2_batch_frames(step: int, batch: int = C2_BATCH, frames: int = C2_STREAM_FRAMES) -> list[int]:
    """Stream frame indices of C2 step `step`: the batch starts where the previous one ended, so
    every frame of the stream is used once per `frames` pairs processed (384 pairs per step over a
    512-frame stream: steps start at frames 0, 384, 256, 128, 0, ...)."""
    s = (step * batch) % frames
    return [(s + i) % frames for i in range(batch)]
