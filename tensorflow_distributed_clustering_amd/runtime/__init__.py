"""Native runtime: in-tree build of the HIP extension and host-side helpers."""
