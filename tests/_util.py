"""Shared helpers for the test suite (fixtures loading, error norms)."""
import math
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_vector(name):
    """TestDataLoader.loadVector (src/test/java/jwave/TestDataLoader.java:46-80)."""
    vals = []
    with open(os.path.join(GOLDEN, "reference_testdata", name)) as f:
        for line in f:
            line = line.strip()
            if line and not line.startswith("#"):
                vals.append(float(line))
    return np.array(vals)


def clean_signal(n):
    """TestSignalGenerator.generateCleanSignal (src/test/java/jwave/transforms/TestSignalGenerator.java:61-69)."""
    i = np.arange(n, dtype=np.float64)
    return (np.sin(2 * math.pi * i / 32.0) + 0.5 * np.sin(2 * math.pi * i / 8.0)
            + 0.25 * np.cos(2 * math.pi * i / 64.0))


def composite_signal(n):
    """TestSignalGenerator.generateCompositeSignal (:25-34): Random(123456789) noise."""
    import oracle as orc
    noise = np.array(orc.java_random_doubles(123456789, n))
    i = np.arange(n, dtype=np.float64)
    return np.sin(2 * math.pi * i / 32.0) + 0.5 * np.sin(2 * math.pi * i / 8.0) + 0.1 * noise


def mse(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.mean((a - b) ** 2))


def normwise(a, b):
    """max|a-b| / max|b| (the BASELINE's normwise relative error)."""
    a, b = np.asarray(a), np.asarray(b)
    den = float(np.max(np.abs(b)))
    return float(np.max(np.abs(a - b))) / (den if den > 0 else 1.0)


def bits_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))
