"""bench.py's roofline launch duration (CPU): the dispatch-stamped figure when
the operation is one kernel the runtime stamps, else -- an op of several
launches (None) or a runtime that refuses the stamped launch (MosrxError) --
the back-to-back figure, and the line says which (launch timing)."""
import mosrx


def test_kernel_duration_prefers_the_stamped_figure():
    import bench
    vals = iter([0.0171, 0.0168, 0.0170, 0.0169, 0.0172, 0.0167])
    ms, how = bench.kernel_duration(lambda: next(vals), 0.0184)
    assert ms == 0.0169 and how.startswith("dispatch-stamped")    # median of the 5 runs after the probe


def test_kernel_duration_falls_back():
    import bench
    ms, how = bench.kernel_duration(lambda: None, 0.0184)
    assert ms == 0.0184 and how.startswith("HIP events around back-to-back")

    def refused():
        raise mosrx.MosrxError(95, "mosrx_time_op_dispatch")
    ms, how = bench.kernel_duration(refused, 0.0184)
    assert ms == 0.0184 and how.startswith("HIP events around back-to-back")
