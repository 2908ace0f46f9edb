// omg_free_gequad.h — the 89-term Gaussian expansion of 1/r used by the
// free-space Green's function: 1/r ~ sum_g w_g exp(-p_g r^2) on [1e-9, 1]
// (relative accuracy ~1e-8), Beylkin's quadrature as tabulated in the
// reference's bundled PSolver, gequad (poisson_3d_fft/build_kernel.f90:
// 1549-1740).  The numbers define the kernel: any other expansion of 1/r would
// move the result at the 1e-8 level, so they are carried over exactly (as
// hexadecimal literals of the same doubles).
#pragma once

namespace omg {

constexpr double kGequadP[89] = {
    0x1.5844a32549d26p+65, 0x1.7d8321e7bd3bcp+63, 0x1.a51cf78478b14p+62,
    0x1.eac3855704547p+61, 0x1.22dcebfc90d24p+61, 0x1.5b19b5fd3fbd1p+60,
    0x1.9f828bbae9e75p+59, 0x1.f23c32e06ceccp+58, 0x1.2b042228f7d90p+58,
    0x1.6725f88736834p+57, 0x1.af936023f8284p+56, 0x1.0364ebb6b7273p+56,
    0x1.37e4e261c87a0p+55, 0x1.771843298441ep+54, 0x1.c32c0bb323b0dp+53,
    0x1.0f5f52974df48p+53, 0x1.467b772025915p+52, 0x1.88cffcec7650ap+51,
    0x1.d8a53ae995910p+50, 0x1.1c5d37ac5a32dp+50, 0x1.562ef886ae16ep+49,
    0x1.9bc5267e1d73cp+48, 0x1.ef84a839eab72p+47, 0x1.2a278d233c418p+47,
    0x1.66ce178bac3a5p+46, 0x1.afcc1c654a0c0p+45, 0x1.03d23a675bc26p+45,
    0x1.38ae63aefbb0cp+44, 0x1.784c12bbef961p+43, 0x1.c4db897d25e71p+42,
    0x1.107f849347b11p+42, 0x1.47f10214c97e5p+41, 0x1.8aaa8431b395bp+40,
    0x1.daf7ababcc26dp+39, 0x1.1dcdd51497b68p+39, 0x1.57f4cb2052bafp+38,
    0x1.9df0d960d73dap+37, 0x1.f22a55887ab2fp+36, 0x1.2bc37eba3094ap+36,
    0x1.68c1bdbc30761p+35, 0x1.b2290de74394dp+34, 0x1.053ff066e1faap+34,
    0x1.3a6818401b01ep+33, 0x1.7a61217aca41cp+32, 0x1.c75e6fc2ac00ap+31,
    0x1.12030486a97a5p+31, 0x1.49c3f45fd1c0cp+30, 0x1.8cdd08e4a3e45p+29,
    0x1.dd9d2b75fe4f7p+28, 0x1.1f65c0ac5f83cp+28, 0x1.59dff146f5ca0p+27,
    0x1.a040257d82725p+26, 0x1.f4f22495ffa40p+25, 0x1.2d6fe8ae92a0ap+25,
    0x1.6ac5697897d21p+24, 0x1.b495bb0ea3843p+23, 0x1.06b575ce67b83p+23,
    0x1.3c29a6f6882c5p+22, 0x1.7c7e318b61b67p+21, 0x1.c9e99f04ea8b1p+20,
    0x1.138adf8ca7e2bp+20, 0x1.4b9b8e1f57dd9p+19, 0x1.8f149af63fe09p+18,
    0x1.e0483c9a08138p+17, 0x1.2100c8b71e3c0p+17, 0x1.5bce9cc372e0dp+16,
    0x1.a29378f6723f5p+15, 0x1.f7be9b06af8adp+14, 0x1.2f1f08477f05ap+14,
    0x1.6ccc42461ebb0p+13, 0x1.b7062671b3599p+12, 0x1.082d325a39b15p+12,
    0x1.3dedd761cdb3ep+11, 0x1.7e9e64267c3a3p+10, 0x1.cc788c6a88a38p+9,
    0x1.1514f786c23d6p+9, 0x1.4d75d60d092dep+8, 0x1.914f63b376cc1p+7,
    0x1.e2f728e36a656p+6, 0x1.229e2168b0febp+6, 0x1.5dc01046536fep+5,
    0x1.a4ea23e6d0c9bp+4, 0x1.fa8ef070ca5dcp+3, 0x1.30cc3d31b644bp+3,
    0x1.6e3550fb28bdcp+2, 0x1.ae63daf257e53p+1, 0x1.c0f365accd678p+0,
    0x1.4b4b5c2bd5ce3p-1, 0x1.2a0c9524ac310p-4,
};
constexpr double kGequadW[89] = {
    0x1.bc00c20193526p+38, 0x1.52ff4709c090ep+33, 0x1.d4c051f0e1542p+32,
    0x1.13cf8a6cc2748p+32, 0x1.26e686d08b05fp+31, 0x1.44f110d1c1860p+30,
    0x1.148d6cae85df8p+33, 0x1.36e4cb5041317p+32, 0x1.7989b8361f92bp+31,
    0x1.ed34c7334ba98p+26, 0x1.7e004dff3ba6ep+26, 0x1.27fabcc343e48p+26,
    0x1.cac7f665c4f4dp+25, 0x1.63a332eec809dp+25, 0x1.13b9b92b74722p+25,
    0x1.ab9738aad3e31p+24, 0x1.4b94cd2e5171dp+24, 0x1.0125e04338f28p+24,
    0x1.8ede89de82311p+23, 0x1.355cb4f769852p+23, 0x1.dfe5c4a6ea776p+22,
    0x1.743ae2b76bf37p+22, 0x1.20b9675c90640p+22, 0x1.bfe94bff0236dp+21,
    0x1.5b6fe8ab428c9p+21, 0x1.0d80ef95794d2p+21, 0x1.a21b1ea77e6d8p+20,
    0x1.445338fddbfbdp+20, 0x1.f7292415435d9p+19, 0x1.864e269c3d73cp+19,
    0x1.2ec36b5524f30p+19, 0x1.d5b6ad1018b0fp+18, 0x1.6c5ccabb99bd4p+18,
    0x1.1aa4055600692p+18, 0x1.b67f1fc60d6edp+17, 0x1.5425e9b035fb8p+17,
    0x1.07dba0e2be43fp+17, 0x1.995b7159d204cp+16, 0x1.3d8b72216811bp+16,
    0x1.eca619465c488p+15, 0x1.7e27cedf0e5c6p+15, 0x1.2871b261b8abap+15,
    0x1.cbe9b7582e9c1p+14, 0x1.64c30c7f95d14p+14, 0x1.14bef9ce1185ap+14,
    0x1.ad5a4d8d44b04p+13, 0x1.4d0e510aa3d0dp+13, 0x1.025b5f0c7d2edp+13,
    0x1.90d2c89a3882dp+12, 0x1.36ecdd4cde942p+12, 0x1.e2612ef4a29ccp+11,
    0x1.7630957665d08p+11, 0x1.2243e0d7dcc10p+11, 0x1.c253ae3cf17a7p+10,
    0x1.5d5371674971dp+10, 0x1.0efa55e0294cep+10, 0x1.a4676a8cfa749p+9,
    0x1.461d404954c39p+9, 0x1.f9f1c2b0a3410p+8, 0x1.88782820fd882p+8,
    0x1.3071e6f308357p+8, 0x1.d8536beefb90bp+7, 0x1.6e6414213e28bp+7,
    0x1.1c3728ac53ee2p+7, 0x1.b8f0f30c78184p+6, 0x1.560b9b50dd173p+6,
    0x1.0954873219706p+6, 0x1.9ba45830d0ca3p+5, 0x1.3f5143aa5e123p+5,
    0x1.ef6649ebf05f9p+4, 0x1.804a21fae8f57p+4, 0x1.2a19889d990abp+4,
    0x1.ce7b52c8e9dbep+3, 0x1.66c13280b5a3dp+3, 0x1.164ab9b6cbffbp+3,
    0x1.afc04e101d68ap+2, 0x1.4eea9f30cf994p+2, 0x1.03ccdb8048188p+2,
    0x1.931006ca6c52ep+1, 0x1.38a98b58b9e67p+1, 0x1.e51314c62f481p+0,
    0x1.7847c40ae51e0p+0, 0x1.23e3a9c14972ep+0, 0x1.c5035abd3d2dcp-1,
    0x1.62a7ca45ca91fp-1, 0x1.2ba52d5bde3ebp-1, 0x1.27016545b7ca3p-1,
    0x1.318132592639bp-1, 0x1.373c08ceadf07p-1,
};

}  // namespace omg
