"""Aggregator builder configuration tables (compressed_communication/builder_configs.py).

LAGRANGE_MULTIPLIER_VALUES (builder_configs.py:16-28): the rate-distortion
lambda the step-size vote uses for each initial step size.
"""

LAGRANGE_MULTIPLIER_VALUES = {
    0.05: 0.0009897002262,
    0.1: 0.001644543016,
    0.25: 0.008091259179,
    0.5: 0.03430265272,
    1.0: 0.1242374538,
    2.0: 0.3964069686,
    2.5: 0.8184151482,
    3.75: 1.470579658,
    5.0: 2.612412919,
    7.5: 5.035264471,
    10.0: 7.369275916,
}
