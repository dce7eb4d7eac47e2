"""Mirror of the reference's ``misc`` package (same module, class and method names).

Replace ``from misc.X import Y`` with ``from deepmatching_stereo_matching_amd.misc.X import Y``
(or alias the package).  Results live on the GPU; numpy arrays are
produced only where the reference API returns them.
"""
