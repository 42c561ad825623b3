"""Single-device compute ops: HIP kernels (GPU) and native host kernels (CPU)."""
from .knn import (knn_cpu, finalize_cpu, merge_cpu, prepare_dataset, knn_gpu,  # noqa: F401
                  merge_gpu, finalize_gpu, format_report_gpu, DeviceDataset, DeviceResult)
