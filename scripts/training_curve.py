"""Training curve from a run's scalars.jsonl (every 50 iterations: total fps, mean reward, mean
episode length) in the format of profiles/*/training_curve.json.
    python scripts/training_curve.py RUN/scalars.jsonl OUT.json "source description" """
import json
import sys


def main(src, out, source):
    curve = {"source": source, "total_fps": {}, "mean_reward": {}, "mean_episode_length": {}}
    keys = {"Perf/total_fps": "total_fps", "Train/mean_reward": "mean_reward",
            "Train/mean_episode_length": "mean_episode_length"}
    for line in open(src):
        d = json.loads(line)
        it = d.get("step", d.get("it", d.get("iteration")))
        tag, val = d.get("tag"), d.get("value")
        if tag in keys and it is not None and int(it) % 50 == 0:
            curve[keys[tag]][str(int(it))] = val
        for k, name in keys.items():  # flat rows {"it": .., "Perf/total_fps": ..}
            if k in d and it is not None and int(it) % 50 == 0:
                curve[name][str(int(it))] = d[k]
    json.dump(curve, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
