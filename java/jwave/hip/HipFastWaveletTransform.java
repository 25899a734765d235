package jwave.hip;

import java.lang.ref.Cleaner;
import java.lang.ref.Reference;

import jwave.exceptions.JWaveException;
import jwave.transforms.FastWaveletTransform;
import jwave.transforms.wavelets.Wavelet;
import jwave.transforms.wavelets.haar.Haar1Orthogonal;

/**
 * Drop-in for {@link FastWaveletTransform}: the 1-D cascade (FastWaveletTransform.java:71-153)
 * and the 2-D row/column transform (BasicTransform.java:361-474) on the MI355X, bit-identical
 * to the JVM with ARITH_STRICT.  Messages and exception classes are the reference's
 * ("given array length is not 2^p ...", "given level is out of range for given array").
 *
 * <p>The native plan is freed by a {@link Cleaner} once the transform is unreachable; every
 * native call keeps the transform reachable until it returns (reachabilityFence), so the plan
 * cannot be freed under a running call.
 */
public class HipFastWaveletTransform extends FastWaveletTransform {
  static {
    HipEngine.load();
  }

  public static final int ARITH_STRICT = 0, ARITH_FMA = 1;
  private static final int KIND_GENERIC = 0, KIND_HAAR_ORTH = 1; // JW_WAVELET_*

  private static final Cleaner CLEANER = Cleaner.create();

  private final long plan; // immutable; lives as long as the transform
  private final int device; // -1: the calling thread's current device

  public HipFastWaveletTransform(Wavelet w) { this(w, ARITH_STRICT, -1); }

  public HipFastWaveletTransform(Wavelet w, int arith) { this(w, arith, -1); }

  public HipFastWaveletTransform(Wavelet w, int arith, int device) {
    super(w);
    this.device = device;
    final long p = nPlanCreate(w.getScalingDeComposition(), w.getWaveletDeComposition(),
                               w.getScalingReConstruction(), w.getWaveletReConstruction(),
                               w.getMotherWavelength(), w.getTransformWavelength(),
                               // Haar1Orthogonal overrides reverse (Haar1Orthogonal.java:175-207)
                               w instanceof Haar1Orthogonal ? KIND_HAAR_ORTH : KIND_GENERIC, arith);
    plan = p;
    CLEANER.register(this, () -> nPlanDestroy(p)); // the action must not capture this
  }

  private double[] line(int op, double[] x, int level) throws JWaveException {
    try {
      if (device >= 0) HipEngine.setDevice(device);
      return nLine(plan, op, x, level);
    } finally {
      Reference.reachabilityFence(this);
    }
  }

  private double[][] matrix(int op, double[][] x, int lvlM, int lvlN) throws JWaveException {
    try {
      if (device >= 0) HipEngine.setDevice(device);
      return nMatrix(plan, op, x, lvlM, lvlN);
    } finally {
      Reference.reachabilityFence(this);
    }
  }

  @Override
  public double[] forward(double[] arrTime, int level) throws JWaveException {
    return line(0, arrTime, level);
  }

  @Override
  public double[] reverse(double[] arrHilb, int level) throws JWaveException {
    return line(1, arrHilb, level);
  }

  private double[][][] space(int op, double[][][] x, int lvlP, int lvlQ, int lvlR)
      throws JWaveException {
    try {
      if (device >= 0) HipEngine.setDevice(device);
      return nSpace(plan, op, x, lvlP, lvlQ, lvlR);
    } finally {
      Reference.reachabilityFence(this);
    }
  }

  @Override
  public double[][] forward(double[][] matTime, int lvlM, int lvlN) throws JWaveException {
    return matrix(0, matTime, lvlM, lvlN);
  }

  @Override
  public double[][] reverse(double[][] matFreq, int lvlM, int lvlN) throws JWaveException {
    return matrix(1, matFreq, lvlM, lvlN);
  }

  /**
   * 3-D (BasicTransform.java:509-565): the 2-D forward of every slab with (lvlP, lvlQ), then the
   * lines along the first dimension with lvlR.  The no-level overload (:487-495) passes
   * getExponent of the three dimensions and reaches this override.
   */
  @Override
  public double[][][] forward(double[][][] spcTime, int lvlP, int lvlQ, int lvlR)
      throws JWaveException {
    return space(0, spcTime, lvlP, lvlQ, lvlR);
  }

  /** 3-D reverse (BasicTransform.java:602-659), the reference's order. */
  @Override
  public double[][][] reverse(double[][][] spcHilb, int lvlP, int lvlQ, int lvlR)
      throws JWaveException {
    return space(1, spcHilb, lvlP, lvlQ, lvlR);
  }

  static native long nPlanCreate(double[] sD, double[] wD, double[] sR, double[] wR,
                                 int motherWavelength, int transformWavelength, int kind,
                                 int arith);
  static native void nPlanDestroy(long plan);
  // op 0 forward, 1 reverse (FWT); 2, 3 the wavelet packet forward / reverse
  static native double[] nLine(long plan, int op, double[] x, int level) throws JWaveException;
  static native double[][] nMatrix(long plan, int op, double[][] x, int lvlM, int lvlN)
      throws JWaveException;
  // op 0 forward, 1 reverse
  static native double[][][] nSpace(long plan, int op, double[][][] x, int lvlP, int lvlQ,
                                    int lvlR) throws JWaveException;
}
