"""Time comb-table builds per window (k_table_pow2 + run-based k_table_fill)
and check a few entries of each table through verification of known
signatures.  Prints one line per build as it happens."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from minbft_amd.authenticator import Authenticator  # noqa: E402


def main():
    ws = [int(x) for x in sys.argv[1:]] or [8, 16, 20, 24, 26, 29]
    with Authenticator(0) as a:
        for w in ws:
            t = time.perf_counter()
            a.set_generator_window(w)
            print(f"G window {w}: {time.perf_counter() - t:.3f} s", flush=True)
        xy = np.frombuffer(bytes.fromhex(
            "87aba255dafedc48324f76048a5bebbf340836bf1ea25c51db6ff426e750ae91"
            "9b2d041020afbb45d9e82da23264895a91991bd6d030b34890376eb7124c331b"), dtype=np.uint8)
        for w in ws:
            a.clear_keys()
            a.set_key_window(w)
            t = time.perf_counter()
            a.register_points(xy[None, :])
            print(f"Q window {w}: {time.perf_counter() - t:.3f} s", flush=True)


if __name__ == "__main__":
    main()
