package jwave.hip;

import jwave.exceptions.JWaveException;
import jwave.transforms.FastWaveletTransform;
import jwave.transforms.wavelets.Wavelet;
import jwave.transforms.wavelets.haar.Haar1Orthogonal;

/**
 * Drop-in for {@link FastWaveletTransform}: the 1-D cascade (FastWaveletTransform.java:71-153)
 * and the 2-D row/column transform (BasicTransform.java:361-474) on the MI355X, bit-identical
 * to the JVM with ARITH_STRICT.  Messages and exception classes are the reference's
 * ("given array length is not 2^p ...", "given level is out of range for given array").
 */
public class HipFastWaveletTransform extends FastWaveletTransform {
  static {
    HipEngine.load();
  }

  public static final int ARITH_STRICT = 0, ARITH_FMA = 1;
  private static final int KIND_GENERIC = 0, KIND_HAAR_ORTH = 1; // JW_WAVELET_*

  private final long plan; // immutable; lives as long as the transform

  public HipFastWaveletTransform(Wavelet w) { this(w, ARITH_STRICT); }

  public HipFastWaveletTransform(Wavelet w, int arith) {
    super(w);
    plan = nPlanCreate(w.getScalingDeComposition(), w.getWaveletDeComposition(),
                       w.getScalingReConstruction(), w.getWaveletReConstruction(),
                       w.getMotherWavelength(), w.getTransformWavelength(),
                       // Haar1Orthogonal overrides reverse (Haar1Orthogonal.java:175-207)
                       w instanceof Haar1Orthogonal ? KIND_HAAR_ORTH : KIND_GENERIC, arith);
  }

  @Override
  public double[] forward(double[] arrTime, int level) throws JWaveException {
    return nLine(plan, 0, arrTime, level);
  }

  @Override
  public double[] reverse(double[] arrHilb, int level) throws JWaveException {
    return nLine(plan, 1, arrHilb, level);
  }

  @Override
  public double[][] forward(double[][] matTime, int lvlM, int lvlN) throws JWaveException {
    return nMatrix(plan, 0, matTime, lvlM, lvlN);
  }

  @Override
  public double[][] reverse(double[][] matFreq, int lvlM, int lvlN) throws JWaveException {
    return nMatrix(plan, 1, matFreq, lvlM, lvlN);
  }

  @Override
  protected void finalize() throws Throwable {
    try {
      nPlanDestroy(plan);
    } finally {
      super.finalize();
    }
  }

  static native long nPlanCreate(double[] sD, double[] wD, double[] sR, double[] wR,
                                 int motherWavelength, int transformWavelength, int kind,
                                 int arith);
  static native void nPlanDestroy(long plan);
  // op 0 forward, 1 reverse (FWT); 2, 3 the wavelet packet forward / reverse
  static native double[] nLine(long plan, int op, double[] x, int level) throws JWaveException;
  static native double[][] nMatrix(long plan, int op, double[][] x, int lvlM, int lvlN)
      throws JWaveException;
}
