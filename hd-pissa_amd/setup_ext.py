"""Builds the torch binding of the probe queue in-tree: hdpissa_amd/_C*.so (g++, torch headers,
linked against hdpissa_amd/_lib/libhdpissa.so).  Run by the Makefile after the library."""
import os

from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CppExtension

HERE = os.path.dirname(os.path.abspath(__file__))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

setup(
    name="hdpissa_amd_C",
    ext_modules=[CppExtension(
        "hdpissa_amd._C", [os.path.join("csrc_ext", "hdp_torch_ext.cpp")],
        include_dirs=[os.path.join(HERE, "..", "include"), os.path.join(ROCM, "include")],
        define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
        library_dirs=[os.path.join(HERE, "hdpissa_amd", "_lib")],
        libraries=["hdpissa", "c10_hip"],
        extra_compile_args=["-O2", "-g0"],
        extra_link_args=["-Wl,-rpath,$ORIGIN/_lib", "-s"],
    )],
    cmdclass={"build_ext": BuildExtension},
)
