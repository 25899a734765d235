package jwave.hip;

import jwave.datatypes.natives.Complex;
import jwave.exceptions.JWaveException;
import jwave.transforms.FastFourierTransform;

/**
 * Drop-in for {@link FastFourierTransform} (FastFourierTransform.java:55-164): the complex
 * forward / reverse (with the reference's 1/n) run through jw_fft_forward_ex /
 * jw_fft_reverse_ex.  ARITH_STRICT (the default) runs the reference's own radix-2 algorithm
 * with its recurrence twiddles (:172-212), bit-identical for power-of-two lengths; ARITH_FMA
 * uses correctly rounded twiddle tables.  The double[] overloads keep the reference's
 * conversions (real input -> interleaved spectrum, spectrum -> real part).
 */
public class HipFastFourierTransform extends FastFourierTransform {
  static {
    HipEngine.load();
  }

  public static final int ARITH_STRICT = 0, ARITH_FMA = 1;

  private final int arith;
  private final int device; // -1: the calling thread's current device

  public HipFastFourierTransform() { this(ARITH_STRICT, -1); }

  public HipFastFourierTransform(int arith, int device) {
    this.arith = arith;
    this.device = device;
  }

  private double[] fft(double[] reim, int dir) {
    if (device >= 0) HipEngine.setDevice(device);
    return nFFT(reim, dir, arith);
  }

  private static double[] interleave(Complex[] x) {
    double[] r = new double[2 * x.length];
    for (int i = 0; i < x.length; i++) {
      r[2 * i] = x[i].getReal();
      r[2 * i + 1] = x[i].getImag();
    }
    return r;
  }

  private static Complex[] complexes(double[] r) {
    Complex[] c = new Complex[r.length / 2];
    for (int i = 0; i < c.length; i++) c[i] = new Complex(r[2 * i], r[2 * i + 1]);
    return c;
  }

  @Override
  public Complex[] forward(Complex[] x) {
    return complexes(fft(interleave(x), 0));
  }

  @Override
  public Complex[] reverse(Complex[] x) {
    return complexes(fft(interleave(x), 1));
  }

  @Override
  public double[] forward(double[] arrTime) throws JWaveException {
    double[] in = new double[2 * arrTime.length]; // (x, 0) pairs, :55-75
    for (int i = 0; i < arrTime.length; i++) in[2 * i] = arrTime[i];
    return fft(in, 0);
  }

  @Override
  public double[] reverse(double[] arrFreq) throws JWaveException {
    double[] t = fft(arrFreq, 1); // real part only, :84-104
    double[] out = new double[arrFreq.length / 2];
    for (int i = 0; i < out.length; i++) out[i] = t[2 * i];
    return out;
  }

  private static native double[] nFFT(double[] reim, int dir, int arith);
}
