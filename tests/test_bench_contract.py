"""bench.py's arithmetic and JSON contract pieces that do not need a GPU."""
import bench


def test_throughput_counts_every_timed_step():
    # 65536 QPs per rank per step, 3 steps in 2.0 s on 2 ranks
    assert bench.throughput(2, 65536, 3, 2.0) == 2 * 65536 * 3 / 2.0


def test_algorithmic_bytes_survey_values():
    """SURVEY.md 8(d) B_solve figures: N=20 K=0 14,056 B; K=8 22,568 B; K=10 24,696 B; N=40 K=10 50,136 B."""
    def nm(N, K):
        return 13 * N - 5, 21 * N - 5 + K * (N - 1)
    assert bench.algorithmic_bytes(*nm(20, 0), 0, 20) == 14056
    assert bench.algorithmic_bytes(*nm(20, 8), 8, 20) == 22568
    assert bench.algorithmic_bytes(*nm(20, 10), 10, 20) == 24696
    assert bench.algorithmic_bytes(*nm(40, 10), 10, 40) == 50136
