package jwave.hip;

import java.lang.ref.Cleaner;
import java.lang.ref.Reference;

import jwave.exceptions.JWaveException;
import jwave.transforms.WaveletPacketTransform;
import jwave.transforms.wavelets.Wavelet;
import jwave.transforms.wavelets.haar.Haar1Orthogonal;

/**
 * Drop-in for {@link WaveletPacketTransform}: the 1-D packet cascade
 * (WaveletPacketTransform.java:73-191), every packet of every level, on the MI355X through
 * jw_wpt_forward / jw_wpt_reverse; bit-identical to the JVM with ARITH_STRICT.  Messages and
 * exception classes are the reference's.  The inherited 2-D and 3-D methods
 * (BasicTransform.java:361-659) call these overrides line by line, as the reference does.
 *
 * <p>The plan is the FWT plan (same filters, same kernels' filter bank); it is freed by a
 * {@link Cleaner} once the transform is unreachable.
 */
public class HipWaveletPacketTransform extends WaveletPacketTransform {
  static {
    HipEngine.load();
  }

  private static final Cleaner CLEANER = Cleaner.create();

  private final long plan;
  private final int device; // -1: the calling thread's current device

  public HipWaveletPacketTransform(Wavelet w) { this(w, HipFastWaveletTransform.ARITH_STRICT, -1); }

  public HipWaveletPacketTransform(Wavelet w, int arith) { this(w, arith, -1); }

  public HipWaveletPacketTransform(Wavelet w, int arith, int device) {
    super(w);
    this.device = device;
    final long p = HipFastWaveletTransform.nPlanCreate(
        w.getScalingDeComposition(), w.getWaveletDeComposition(), w.getScalingReConstruction(),
        w.getWaveletReConstruction(), w.getMotherWavelength(), w.getTransformWavelength(),
        w instanceof Haar1Orthogonal ? 1 : 0, arith); // JW_WAVELET_HAAR_ORTH / GENERIC
    plan = p;
    CLEANER.register(this, () -> HipFastWaveletTransform.nPlanDestroy(p));
  }

  private double[] line(int op, double[] x, int level) throws JWaveException {
    try {
      if (device >= 0) HipEngine.setDevice(device);
      return HipFastWaveletTransform.nLine(plan, op, x, level);
    } finally {
      Reference.reachabilityFence(this);
    }
  }

  @Override
  public double[] forward(double[] arrTime, int level) throws JWaveException {
    return line(2, arrTime, level);
  }

  @Override
  public double[] reverse(double[] arrHilb, int level) throws JWaveException {
    return line(3, arrHilb, level);
  }
}
