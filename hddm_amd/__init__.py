"""hddm_amd — MI355X-native WFPT likelihood engine for HDDM.

`hddm_amd.wfpt` is the drop-in for the reference's `wfpt` extension module
(src/wfpt.pyx); `hddm_amd.likelihoods` carries the PyMC-facing `wfpt_like`
(hddm/likelihoods.py:52-73). All densities come from the HIP kernels in
hddm_amd/csrc (libwfpt_amd.so); importing `hddm_amd.wfpt` without the built
library raises ImportError.
"""
__version__ = "0.1.0"
