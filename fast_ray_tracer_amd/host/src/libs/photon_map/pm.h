/*
 * frt-mi355x host API: photon map (Jensen kd-tree) storage.
 * Struct layout follows reference src/libs/photon_map/pm.h:5-42 so that
 * generated main.c (array_of_photon_maps / init_Photon_map) compiles.
 */
#ifndef FRT_PM_H
#define FRT_PM_H

typedef struct Photon {
    double pos[3];
    short plane;
    unsigned char theta, phi;
    double power[3];
} Photon;

typedef struct NearestPhotons {
    long max;
    long found;
    int got_heap;
    double pos[3];
    double *dist2;
    Photon **index;
} NearestPhotons;

typedef struct {
    Photon *photons;
    long stored_photons;
    long half_stored_photons;
    long max_photons;
    long prev_scale;
    double costheta[256];
    double sintheta[256];
    double cosphi[256];
    double sinphi[256];
    double bbox_min[3];
    double bbox_max[3];
} PhotonMap;

void init_Photon_map(long max_phot, PhotonMap *pm);
void delete_Photon_map(PhotonMap *pm);
void pm_store(PhotonMap *pm, double power[3], double pos[3], double dir[3]);
void pm_scale_photon_power(PhotonMap *pm, double scale);
void pm_balance(PhotonMap *pm);

#endif
