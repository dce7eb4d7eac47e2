"""Sample the GPU's socket power and shader clock (rocm-smi, sysfs: no HIP) while a command runs.

    python tools/power_watch.py OUT.jsonl -- python3 bench.py --steps 2000 --no-volume ...

Starts the command as a child process, samples every ~0.5 s until it exits, writes one JSON
object per sample and returns the command's exit status.  Used to see whether the level
kernel's clock under load is set by the power cap (DVFS).
"""
import json
import subprocess
import sys
import time


def sample():
    try:
        out = subprocess.run(['rocm-smi', '--showpower', '--showclocks', '--showtemp', '--json'],
                             capture_output=True, text=True, timeout=10).stdout
        return json.loads(out[out.index('{'):])
    except Exception as e:  # noqa: BLE001 -- a failed sample is recorded, not fatal
        return {'error': repr(e)}


def main():
    out = sys.argv[1]
    cmd = sys.argv[sys.argv.index('--') + 1:]
    t0 = time.time()
    p = subprocess.Popen(cmd)
    with open(out, 'w') as f:
        while p.poll() is None:
            f.write(json.dumps({'t': round(time.time() - t0, 2), 's': sample()}) + '\n')
            f.flush()
            time.sleep(0.5)
    sys.exit(p.returncode)


if __name__ == '__main__':
    main()
