"""Native (C++) runtime components built in-tree by ``kubeoperator_amd.ops._build.build_native``:

* ``prefetch`` -- multi-threaded token-window prefetcher over a memory-mapped token file.
"""
