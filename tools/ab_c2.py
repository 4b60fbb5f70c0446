"""Same-box A/B of the C2 leg (tools/build_ab.sh): for each library given, alternating, (1) every
extraction / stereo kernel's duration with one engine and nothing else on the GPU (128 pairs, the
engine profiler's hipEvents) and (2) the pipelined C2 leg's stereo frames/s (3 engines x 128 pairs
over bench.py's 512-frame stream, bench.py's own timing). Each measurement runs in a fresh process
with ORBSLAM_AMD_LIB set; the stream is generated once (cached in $TMPDIR).
  python tools/ab_c2.py <lib_a.so> <lib_b.so> [rounds]"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

CHILD = r'''
import json, sys, time
import numpy as np
sys.path.insert(0, "ROOT/orb-slam2-noted_amd/python"); sys.path.insert(0, "ROOT")
import bench   # sets GPU_MAX_HW_QUEUES before the runtime starts, as bench.py does
import torch
torch.cuda.init()
import orbslam2_amd as amd
st = np.load("STREAM", mmap_mode="r")   # [512][2][376][1241]
pool = [(st[t, 0], st[t, 1]) for t in range(len(st))]
B = 128
imgs = np.ascontiguousarray(st[:B]).reshape(2 * B, 376, 1241)
d = torch.from_numpy(imgs).cuda()
torch.cuda.synchronize()
mb = float(np.float32(386.1448) / np.float32(718.856))
pl = amd.StereoPipeline(2000, n_engines=1)
pl.reserve(1241, 376, B)
for _ in range(3):
    pl.stereo_batch(d.data_ptr(), B, 1241, 376, 1241, 1241 * 376, 386.1448, mb)
amd.device_sync()
pl.profile(True)
for _ in range(5):
    pl.stereo_batch(d.data_ptr(), B, 1241, 376, 1241, 1241 * 376, 386.1448, mb)
    amd.device_sync()
iso = {k: round(v[0] / 5, 4) for k, v in pl.profile_read().items()}
pl.close()
class A: pass
args = A(); args.batch = 384; args.engines = 3; args.warmup = 3; args.steps = 30; args.blur_mode = 0
buf = bench.c2_stream_buffer(pool)
params = (2000, 1.2, 8, 20, 7, 386.1448, mb)
el, _, ex = bench.time_c2(amd, args, None, params, buf, 0, args.steps)
ex.close()
print(json.dumps({"iso_ms": iso, "iso_total_ms": round(sum(iso.values()), 4), "c2": round(384 * 30 / el, 1)}))
'''.replace("ROOT", str(ROOT))


STREAM = Path(os.environ.get("TMPDIR", "/tmp")) / "ab_c2_stream.npy"


def stream_file():
    if not STREAM.exists():
        sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))
        import numpy as np
        from orbslam2_amd import synth
        np.save(STREAM, np.stack([np.stack(p) for p in synth.stereo_stream(376, 1241, 512)]))
    return STREAM


def run(lib):
    env = dict(os.environ, ORBSLAM_AMD_LIB=str(Path(lib).resolve()))
    r = subprocess.run([sys.executable, "-c", CHILD.replace("STREAM", str(stream_file()))], env=env, capture_output=True, text=True, timeout=300)
    if r.returncode:
        raise SystemExit(r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    libs = sys.argv[1:3]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    res = {l: [] for l in libs}
    for r in range(rounds):
        for l in (libs if r % 2 == 0 else libs[::-1]):
            o = run(l)
            res[l].append(o)
            print(Path(l).parent.name, json.dumps(o), flush=True)
    for l in libs:
        c2 = [o["c2"] for o in res[l]]
        iso = {k: round(sum(o["iso_ms"].get(k, 0) for o in res[l]) / len(res[l]), 4) for k in res[l][0]["iso_ms"]}
        print("SUMMARY", Path(l).parent.name, "c2 mean", round(sum(c2) / len(c2), 1), "runs", c2, "iso", json.dumps(iso),
              flush=True)


if __name__ == "__main__":
    main()
