#!/usr/bin/env python3
"""generate_input.py-compatible workload generator (same CLI, byte-identical output for the same
seed: same `random` call sequence as the reference's generate_input.py:6-23).  --fast switches
to the vectorised numpy generator (same distribution, different stream) for large inputs."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_machine_learning_project_amd.utils.io import generate, generate_text, to_text  # noqa: E402


def main():
    p = argparse.ArgumentParser(description="Generate input for the k-NN engine.")
    p.add_argument("--num_data", type=int, required=True)
    p.add_argument("--num_queries", type=int, required=True)
    p.add_argument("--num_attrs", type=int, required=True)
    p.add_argument("--min", type=float, required=True)
    p.add_argument("--max", type=float, required=True)
    p.add_argument("--minK", type=int, required=True)
    p.add_argument("--maxK", type=int, required=True)
    p.add_argument("--num_labels", type=int, required=True)
    p.add_argument("--output", type=str, required=True)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--fast", action="store_true", help="numpy generator (large N)")
    a = p.parse_args()
    if a.min >= a.max:
        sys.exit("Error: --min must be less than --max")
    if a.minK > a.maxK:
        sys.exit("Error: --minK must be ≤ --maxK")
    if a.num_labels <= 0:
        sys.exit("Error: --num_labels must be positive")
    if a.fast:
        text = to_text(generate(a.num_data, a.num_queries, a.num_attrs, a.min, a.max, a.minK,
                                a.maxK, a.num_labels, a.seed))
    else:
        text = generate_text(a.num_data, a.num_queries, a.num_attrs, a.min, a.max, a.minK, a.maxK,
                             a.num_labels, a.seed)
    with open(a.output, "w") as f:
        f.write(text)
    print(f"✅ Input file '{a.output}' generated successfully.")


if __name__ == "__main__":
    main()
