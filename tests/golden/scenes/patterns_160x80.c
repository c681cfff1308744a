#include <stdio.h>
#include <string.h>
#include <stdbool.h>
#include <math.h>
#include <unistd.h>

#include "src/libs/canvas/canvas.h"
#include "src/libs/linalg/linalg.h"
#include "src/libs/obj_loader/obj_loader.h"
#include "src/libs/photon_map/pm.h"
#include "src/color/hsl.h"
#include "src/color/lab.h"
#include "src/color/rgb.h"
#include "src/color/srgb.h"
#include "src/color/xyz.h"
#include "src/color/xyy.h"

#include "src/renderer/camera.h"
#include "src/renderer/config.h"
#include "src/renderer/photon_tracer.h"
#include "src/renderer/renderer.h"
#include "src/renderer/world.h"
#include "src/pattern/pattern.h"
#include "src/shapes/shapes.h"
#include "src/shapes/cone.h"
#include "src/shapes/csg.h"
#include "src/shapes/cube.h"
#include "src/shapes/cylinder.h"
#include "src/shapes/group.h"
#include "src/shapes/plane.h"
#include "src/shapes/sphere.h"
#include "src/shapes/triangle.h"
#include "src/shapes/toroid.h"

#define True true
#define False false

int
main()
{
    /* config */
    struct global_config global_config;
    global_config.illumination.include_direct = True;
    global_config.illumination.include_global = False;
    global_config.illumination.debug_visualize_photon_map = False;
    global_config.illumination.debug_visualize_soft_indirect = False;
    global_config.illumination.di.include_ambient = True;
    global_config.illumination.di.include_diffuse = True;
    global_config.illumination.di.include_specular_highlight = True;
    global_config.illumination.di.include_specular = True;
    global_config.illumination.di.path_length = 5;

    global_config.illumination.gi.include_caustics = False;
    global_config.illumination.gi.include_final_gather = False;
    global_config.illumination.gi.usteps = 1;
    global_config.illumination.gi.vsteps = 1;
    global_config.illumination.gi.irradiance_estimate_num = 200;
    global_config.illumination.gi.irradiance_estimate_radius = 0.1000000000;
    global_config.illumination.gi.irradiance_estimate_cone_filter_k = 1.0000000000;
    global_config.illumination.gi.photon_count = 0;
    global_config.illumination.gi.path_length = 5;

    global_config.threading.num_threads = 1;
    global_config.scene.divide_threshold = 1;
    global_config.output.file_path = "/tmp/frt_golden/out/patterns_160x80";
    global_config.output.color_space = SRGB;

    void (*color_space_fn)(const Color, Color) = NULL;
    switch (global_config.output.color_space) {
    case RGB:
        color_space_fn = rgb_to_rgb;
        break;
    case HSL:
        color_space_fn = hsl_to_rgb;
        break;
    case XYZ:
        color_space_fn = xyz_to_rgb;
        break;
    case XYY:
        color_space_fn = xyy_to_rgb;
        break;
    case LAB:
        color_space_fn = lab_to_rgb;
        break;
    case SRGB:
        // this is the default
    default:
        color_space_fn = srgb_to_rgb;
        break;
    }

    /* end config */

    /* camera */
    struct aperture ap;
    aperture(POINT_APERTURE, 0.0, 1, 1, false, &ap);

    Point from = { 0.0000000000, 2.2000000000, -6.0000000000, 1.0 };
    Point to = { 0.0000000000, 0.6000000000, 0.0000000000, 1.0 };
    Vector up = { 0.0000000000, 1.0000000000, 0.0000000000, 0.0 };
    Matrix camera_xform;
    view_transform(from, to, up, camera_xform);

    Camera cam = camera(160, 80, 1.0000000000/*field_of_view*/, 1.0000000000/*distance*/, 1/*usteps*/, 1/*vsteps*/, &ap, camera_xform);

    /* end camera */

    /* lights */
    Light all_lights = array_of_lights(1);

    /* point light 0 */
    Light point_light_0 = all_lights + 0;
    Point point_light_0_point = { -6.0000000000, 8.0000000000, -8.0000000000, 1.0 };
    Color point_light_0_intensity = color(1.0000000000, 1.0000000000, 1.0000000000);
    point_light(point_light_0_point, point_light_0_intensity, point_light_0);

    /* end point light 0 */

    /* end lights */

    /* shapes */
    Shape all_shapes = array_of_shapes(4);

    /* shape 0 */
    
    Matrix transform_pattern_0_Ka;
    matrix_identity(transform_pattern_0_Ka);
    Matrix transform_pattern_blended_0_Ka_0;
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_pattern_blended_0_Ka_0);
    Color pattern_blended_0_Ka_0_color_0_raw = color(0.9000000000, 0.2000000000, 0.2000000000);
    Color pattern_blended_0_Ka_0_color_1_raw = color(0.9500000000, 0.9500000000, 0.9500000000);
    Color pattern_blended_0_Ka_0_color_0;
    Color pattern_blended_0_Ka_0_color_1;
    color_space_fn(pattern_blended_0_Ka_0_color_0_raw, pattern_blended_0_Ka_0_color_0);
    color_space_fn(pattern_blended_0_Ka_0_color_1_raw, pattern_blended_0_Ka_0_color_1);
    Pattern pattern_blended_0_Ka_0 = stripe_pattern_alloc(pattern_blended_0_Ka_0_color_0, pattern_blended_0_Ka_0_color_1);

    pattern_set_transform(pattern_blended_0_Ka_0, transform_pattern_blended_0_Ka_0);

Matrix transform_pattern_blended_0_Ka_1, transform_pattern_blended_0_Ka_1_tmp;
    matrix_identity(transform_pattern_blended_0_Ka_1);
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_pattern_blended_0_Ka_1_tmp);
    transform_chain(transform_pattern_blended_0_Ka_1_tmp, transform_pattern_blended_0_Ka_1);
    matrix_rotate_y(1.5707963000, transform_pattern_blended_0_Ka_1_tmp);
    transform_chain(transform_pattern_blended_0_Ka_1_tmp, transform_pattern_blended_0_Ka_1);

    Color pattern_blended_0_Ka_1_color_0_raw = color(0.2000000000, 0.2000000000, 0.9000000000);
    Color pattern_blended_0_Ka_1_color_1_raw = color(0.9500000000, 0.9500000000, 0.9500000000);
    Color pattern_blended_0_Ka_1_color_0;
    Color pattern_blended_0_Ka_1_color_1;
    color_space_fn(pattern_blended_0_Ka_1_color_0_raw, pattern_blended_0_Ka_1_color_0);
    color_space_fn(pattern_blended_0_Ka_1_color_1_raw, pattern_blended_0_Ka_1_color_1);
    Pattern pattern_blended_0_Ka_1 = stripe_pattern_alloc(pattern_blended_0_Ka_1_color_0, pattern_blended_0_Ka_1_color_1);

    pattern_set_transform(pattern_blended_0_Ka_1, transform_pattern_blended_0_Ka_1);

    Pattern pattern_0_Ka = blended_pattern_alloc(pattern_blended_0_Ka_0, pattern_blended_0_Ka_1);
    pattern_set_transform(pattern_0_Ka, transform_pattern_0_Ka);
Matrix transform_pattern_0_Kd;
    matrix_identity(transform_pattern_0_Kd);
    Matrix transform_pattern_blended_0_Kd_0;
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_pattern_blended_0_Kd_0);
    Color pattern_blended_0_Kd_0_color_0_raw = color(0.9000000000, 0.2000000000, 0.2000000000);
    Color pattern_blended_0_Kd_0_color_1_raw = color(0.9500000000, 0.9500000000, 0.9500000000);
    Color pattern_blended_0_Kd_0_color_0;
    Color pattern_blended_0_Kd_0_color_1;
    color_space_fn(pattern_blended_0_Kd_0_color_0_raw, pattern_blended_0_Kd_0_color_0);
    color_space_fn(pattern_blended_0_Kd_0_color_1_raw, pattern_blended_0_Kd_0_color_1);
    Pattern pattern_blended_0_Kd_0 = stripe_pattern_alloc(pattern_blended_0_Kd_0_color_0, pattern_blended_0_Kd_0_color_1);

    pattern_set_transform(pattern_blended_0_Kd_0, transform_pattern_blended_0_Kd_0);

Matrix transform_pattern_blended_0_Kd_1, transform_pattern_blended_0_Kd_1_tmp;
    matrix_identity(transform_pattern_blended_0_Kd_1);
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_pattern_blended_0_Kd_1_tmp);
    transform_chain(transform_pattern_blended_0_Kd_1_tmp, transform_pattern_blended_0_Kd_1);
    matrix_rotate_y(1.5707963000, transform_pattern_blended_0_Kd_1_tmp);
    transform_chain(transform_pattern_blended_0_Kd_1_tmp, transform_pattern_blended_0_Kd_1);

    Color pattern_blended_0_Kd_1_color_0_raw = color(0.2000000000, 0.2000000000, 0.9000000000);
    Color pattern_blended_0_Kd_1_color_1_raw = color(0.9500000000, 0.9500000000, 0.9500000000);
    Color pattern_blended_0_Kd_1_color_0;
    Color pattern_blended_0_Kd_1_color_1;
    color_space_fn(pattern_blended_0_Kd_1_color_0_raw, pattern_blended_0_Kd_1_color_0);
    color_space_fn(pattern_blended_0_Kd_1_color_1_raw, pattern_blended_0_Kd_1_color_1);
    Pattern pattern_blended_0_Kd_1 = stripe_pattern_alloc(pattern_blended_0_Kd_1_color_0, pattern_blended_0_Kd_1_color_1);

    pattern_set_transform(pattern_blended_0_Kd_1, transform_pattern_blended_0_Kd_1);

    Pattern pattern_0_Kd = blended_pattern_alloc(pattern_blended_0_Kd_0, pattern_blended_0_Kd_1);
    pattern_set_transform(pattern_0_Kd, transform_pattern_0_Kd);
    Pattern pattern_0_Ks = NULL;
    Pattern pattern_0_Ns = NULL;
    Pattern pattern_0_bump = NULL;
    Pattern pattern_0_disp = NULL;
    Pattern pattern_0_refl = NULL;
    Pattern pattern_0_d = NULL;
    Color material_0_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_0_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_0 = material_alloc();
    color_space_fn(material_0_color_raw, material_0->Ka);
    color_space_fn(material_0_color_raw, material_0->Kd);
    color_space_fn(material_0_color_raw, material_0->Ks);
    color_scale(material_0->Ka, 0.1500000000);
    color_scale(material_0->Kd, 0.8000000000);
    color_scale(material_0->Ks, 0.1000000000);
    rgb_to_rgb(material_0_reflective, material_0->refl);
    rgb_to_rgb(material_0_refractive, material_0->Tf);
    material_0->reflective = material_0_reflective[0] > 0.0
                             || material_0_reflective[1] > 0.0
                             || material_0_reflective[2] > 0.0;

    material_0->Tr = 0.0000000000;
    material_0->Ns = 200.0000000000;
    material_0->Ni = 1.0000000000;
    material_0->casts_shadow = true;
    material_set_pattern(material_0, map_Ka, pattern_0_Ka);
    material_set_pattern(material_0, map_Kd, pattern_0_Kd);
    material_set_pattern(material_0, map_Ks, pattern_0_Ks);
    material_set_pattern(material_0, map_Ns, pattern_0_Ns);
    material_set_pattern(material_0, map_d, pattern_0_d);
    material_set_pattern(material_0, map_bump, pattern_0_bump);
    material_set_pattern(material_0, map_disp, pattern_0_disp);
    material_set_pattern(material_0, map_refl, pattern_0_refl);

    Matrix transform_0;
    matrix_identity(transform_0);
    Shape shape_0 = all_shapes + 0;
    plane(shape_0);
    shape_set_material(shape_0, material_0);
    shape_set_transform(shape_0, transform_0);

    /* end shape 0 */
    /* shape 1 */
    
    Matrix transform_pattern_1_Ka;
    matrix_identity(transform_pattern_1_Ka);
    Matrix transform_pattern_nested_1_Ka_0;
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_pattern_nested_1_Ka_0);
    Color pattern_nested_1_Ka_0_color_0_raw = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_nested_1_Ka_0_color_1_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_nested_1_Ka_0_color_0;
    Color pattern_nested_1_Ka_0_color_1;
    color_space_fn(pattern_nested_1_Ka_0_color_0_raw, pattern_nested_1_Ka_0_color_0);
    color_space_fn(pattern_nested_1_Ka_0_color_1_raw, pattern_nested_1_Ka_0_color_1);
    Pattern pattern_nested_1_Ka_0 = checker_pattern_alloc(pattern_nested_1_Ka_0_color_0, pattern_nested_1_Ka_0_color_1);

    pattern_set_transform(pattern_nested_1_Ka_0, transform_pattern_nested_1_Ka_0);

Matrix transform_pattern_nested_1_Ka_1;
    matrix_scale(0.1500000000, 0.1500000000, 0.1500000000, transform_pattern_nested_1_Ka_1);
    Color pattern_nested_1_Ka_1_color_0_raw = color(0.1000000000, 0.6000000000, 0.1000000000);
    Color pattern_nested_1_Ka_1_color_1_raw = color(0.9000000000, 0.9000000000, 0.2000000000);
    Color pattern_nested_1_Ka_1_color_0;
    Color pattern_nested_1_Ka_1_color_1;
    color_space_fn(pattern_nested_1_Ka_1_color_0_raw, pattern_nested_1_Ka_1_color_0);
    color_space_fn(pattern_nested_1_Ka_1_color_1_raw, pattern_nested_1_Ka_1_color_1);
    Pattern pattern_nested_1_Ka_1 = stripe_pattern_alloc(pattern_nested_1_Ka_1_color_0, pattern_nested_1_Ka_1_color_1);

    pattern_set_transform(pattern_nested_1_Ka_1, transform_pattern_nested_1_Ka_1);

Matrix transform_pattern_nested_1_Ka_2;
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_pattern_nested_1_Ka_2);
    Color pattern_nested_1_Ka_2_color_0_raw = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_nested_1_Ka_2_color_1_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_nested_1_Ka_2_color_0;
    Color pattern_nested_1_Ka_2_color_1;
    color_space_fn(pattern_nested_1_Ka_2_color_0_raw, pattern_nested_1_Ka_2_color_0);
    color_space_fn(pattern_nested_1_Ka_2_color_1_raw, pattern_nested_1_Ka_2_color_1);
    Pattern pattern_nested_1_Ka_2 = checker_pattern_alloc(pattern_nested_1_Ka_2_color_0, pattern_nested_1_Ka_2_color_1);

    pattern_set_transform(pattern_nested_1_Ka_2, transform_pattern_nested_1_Ka_2);

    Pattern pattern_1_Ka = nested_pattern_alloc(pattern_nested_1_Ka_0, pattern_nested_1_Ka_1, pattern_nested_1_Ka_2);
    pattern_set_transform(pattern_1_Ka, transform_pattern_1_Ka);
Matrix transform_pattern_1_Kd;
    matrix_identity(transform_pattern_1_Kd);
    Matrix transform_pattern_nested_1_Kd_0;
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_pattern_nested_1_Kd_0);
    Color pattern_nested_1_Kd_0_color_0_raw = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_nested_1_Kd_0_color_1_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_nested_1_Kd_0_color_0;
    Color pattern_nested_1_Kd_0_color_1;
    color_space_fn(pattern_nested_1_Kd_0_color_0_raw, pattern_nested_1_Kd_0_color_0);
    color_space_fn(pattern_nested_1_Kd_0_color_1_raw, pattern_nested_1_Kd_0_color_1);
    Pattern pattern_nested_1_Kd_0 = checker_pattern_alloc(pattern_nested_1_Kd_0_color_0, pattern_nested_1_Kd_0_color_1);

    pattern_set_transform(pattern_nested_1_Kd_0, transform_pattern_nested_1_Kd_0);

Matrix transform_pattern_nested_1_Kd_1;
    matrix_scale(0.1500000000, 0.1500000000, 0.1500000000, transform_pattern_nested_1_Kd_1);
    Color pattern_nested_1_Kd_1_color_0_raw = color(0.1000000000, 0.6000000000, 0.1000000000);
    Color pattern_nested_1_Kd_1_color_1_raw = color(0.9000000000, 0.9000000000, 0.2000000000);
    Color pattern_nested_1_Kd_1_color_0;
    Color pattern_nested_1_Kd_1_color_1;
    color_space_fn(pattern_nested_1_Kd_1_color_0_raw, pattern_nested_1_Kd_1_color_0);
    color_space_fn(pattern_nested_1_Kd_1_color_1_raw, pattern_nested_1_Kd_1_color_1);
    Pattern pattern_nested_1_Kd_1 = stripe_pattern_alloc(pattern_nested_1_Kd_1_color_0, pattern_nested_1_Kd_1_color_1);

    pattern_set_transform(pattern_nested_1_Kd_1, transform_pattern_nested_1_Kd_1);

Matrix transform_pattern_nested_1_Kd_2;
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_pattern_nested_1_Kd_2);
    Color pattern_nested_1_Kd_2_color_0_raw = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_nested_1_Kd_2_color_1_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_nested_1_Kd_2_color_0;
    Color pattern_nested_1_Kd_2_color_1;
    color_space_fn(pattern_nested_1_Kd_2_color_0_raw, pattern_nested_1_Kd_2_color_0);
    color_space_fn(pattern_nested_1_Kd_2_color_1_raw, pattern_nested_1_Kd_2_color_1);
    Pattern pattern_nested_1_Kd_2 = checker_pattern_alloc(pattern_nested_1_Kd_2_color_0, pattern_nested_1_Kd_2_color_1);

    pattern_set_transform(pattern_nested_1_Kd_2, transform_pattern_nested_1_Kd_2);

    Pattern pattern_1_Kd = nested_pattern_alloc(pattern_nested_1_Kd_0, pattern_nested_1_Kd_1, pattern_nested_1_Kd_2);
    pattern_set_transform(pattern_1_Kd, transform_pattern_1_Kd);
    Pattern pattern_1_Ks = NULL;
    Pattern pattern_1_Ns = NULL;
    Pattern pattern_1_bump = NULL;
    Pattern pattern_1_disp = NULL;
    Pattern pattern_1_refl = NULL;
    Pattern pattern_1_d = NULL;
    Color material_1_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_1_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_1_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_1 = material_alloc();
    color_space_fn(material_1_color_raw, material_1->Ka);
    color_space_fn(material_1_color_raw, material_1->Kd);
    color_space_fn(material_1_color_raw, material_1->Ks);
    color_scale(material_1->Ka, 0.1000000000);
    color_scale(material_1->Kd, 0.7000000000);
    color_scale(material_1->Ks, 0.3000000000);
    rgb_to_rgb(material_1_reflective, material_1->refl);
    rgb_to_rgb(material_1_refractive, material_1->Tf);
    material_1->reflective = material_1_reflective[0] > 0.0
                             || material_1_reflective[1] > 0.0
                             || material_1_reflective[2] > 0.0;

    material_1->Tr = 0.0000000000;
    material_1->Ns = 50.0000000000;
    material_1->Ni = 1.0000000000;
    material_1->casts_shadow = true;
    material_set_pattern(material_1, map_Ka, pattern_1_Ka);
    material_set_pattern(material_1, map_Kd, pattern_1_Kd);
    material_set_pattern(material_1, map_Ks, pattern_1_Ks);
    material_set_pattern(material_1, map_Ns, pattern_1_Ns);
    material_set_pattern(material_1, map_d, pattern_1_d);
    material_set_pattern(material_1, map_bump, pattern_1_bump);
    material_set_pattern(material_1, map_disp, pattern_1_disp);
    material_set_pattern(material_1, map_refl, pattern_1_refl);

    Matrix transform_1;
    matrix_translate(-2.2000000000, 1.0000000000, 0.5000000000, transform_1);
    Shape shape_1 = all_shapes + 1;
    sphere(shape_1);
    shape_set_material(shape_1, material_1);
    shape_set_transform(shape_1, transform_1);

    /* end shape 1 */
    /* shape 2 */
    
    Matrix transform_pattern_2_Ka;
    matrix_identity(transform_pattern_2_Ka);
    Matrix transform_pattern_perturbed_2_Ka_0;
    matrix_scale(0.1000000000, 0.1000000000, 0.1000000000, transform_pattern_perturbed_2_Ka_0);
    Color pattern_perturbed_2_Ka_0_color_0_raw = color(0.8000000000, 0.5000000000, 0.2000000000);
    Color pattern_perturbed_2_Ka_0_color_1_raw = color(0.3000000000, 0.1500000000, 0.0500000000);
    Color pattern_perturbed_2_Ka_0_color_0;
    Color pattern_perturbed_2_Ka_0_color_1;
    color_space_fn(pattern_perturbed_2_Ka_0_color_0_raw, pattern_perturbed_2_Ka_0_color_0);
    color_space_fn(pattern_perturbed_2_Ka_0_color_1_raw, pattern_perturbed_2_Ka_0_color_1);
    Pattern pattern_perturbed_2_Ka_0 = ring_pattern_alloc(pattern_perturbed_2_Ka_0_color_0, pattern_perturbed_2_Ka_0_color_1);

    pattern_set_transform(pattern_perturbed_2_Ka_0, transform_pattern_perturbed_2_Ka_0);

    Pattern pattern_2_Ka = perturbed_pattern_alloc(pattern_perturbed_2_Ka_0, 2.0000000000, 0.3000000000, 0.6000000000, 3, 7);
    pattern_set_transform(pattern_2_Ka, transform_pattern_2_Ka);
Matrix transform_pattern_2_Kd;
    matrix_identity(transform_pattern_2_Kd);
    Matrix transform_pattern_perturbed_2_Kd_0;
    matrix_scale(0.1000000000, 0.1000000000, 0.1000000000, transform_pattern_perturbed_2_Kd_0);
    Color pattern_perturbed_2_Kd_0_color_0_raw = color(0.8000000000, 0.5000000000, 0.2000000000);
    Color pattern_perturbed_2_Kd_0_color_1_raw = color(0.3000000000, 0.1500000000, 0.0500000000);
    Color pattern_perturbed_2_Kd_0_color_0;
    Color pattern_perturbed_2_Kd_0_color_1;
    color_space_fn(pattern_perturbed_2_Kd_0_color_0_raw, pattern_perturbed_2_Kd_0_color_0);
    color_space_fn(pattern_perturbed_2_Kd_0_color_1_raw, pattern_perturbed_2_Kd_0_color_1);
    Pattern pattern_perturbed_2_Kd_0 = ring_pattern_alloc(pattern_perturbed_2_Kd_0_color_0, pattern_perturbed_2_Kd_0_color_1);

    pattern_set_transform(pattern_perturbed_2_Kd_0, transform_pattern_perturbed_2_Kd_0);

    Pattern pattern_2_Kd = perturbed_pattern_alloc(pattern_perturbed_2_Kd_0, 2.0000000000, 0.3000000000, 0.6000000000, 3, 7);
    pattern_set_transform(pattern_2_Kd, transform_pattern_2_Kd);
    Pattern pattern_2_Ks = NULL;
    Pattern pattern_2_Ns = NULL;
    Pattern pattern_2_bump = NULL;
    Pattern pattern_2_disp = NULL;
    Pattern pattern_2_refl = NULL;
    Pattern pattern_2_d = NULL;
    Color material_2_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_2_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_2_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_2 = material_alloc();
    color_space_fn(material_2_color_raw, material_2->Ka);
    color_space_fn(material_2_color_raw, material_2->Kd);
    color_space_fn(material_2_color_raw, material_2->Ks);
    color_scale(material_2->Ka, 0.1000000000);
    color_scale(material_2->Kd, 0.7000000000);
    color_scale(material_2->Ks, 0.3000000000);
    rgb_to_rgb(material_2_reflective, material_2->refl);
    rgb_to_rgb(material_2_refractive, material_2->Tf);
    material_2->reflective = material_2_reflective[0] > 0.0
                             || material_2_reflective[1] > 0.0
                             || material_2_reflective[2] > 0.0;

    material_2->Tr = 0.0000000000;
    material_2->Ns = 50.0000000000;
    material_2->Ni = 1.0000000000;
    material_2->casts_shadow = true;
    material_set_pattern(material_2, map_Ka, pattern_2_Ka);
    material_set_pattern(material_2, map_Kd, pattern_2_Kd);
    material_set_pattern(material_2, map_Ks, pattern_2_Ks);
    material_set_pattern(material_2, map_Ns, pattern_2_Ns);
    material_set_pattern(material_2, map_d, pattern_2_d);
    material_set_pattern(material_2, map_bump, pattern_2_bump);
    material_set_pattern(material_2, map_disp, pattern_2_disp);
    material_set_pattern(material_2, map_refl, pattern_2_refl);

    Matrix transform_2;
    matrix_translate(0.0000000000, 1.0000000000, 0.0000000000, transform_2);
    Shape shape_2 = all_shapes + 2;
    sphere(shape_2);
    shape_set_material(shape_2, material_2);
    shape_set_transform(shape_2, transform_2);

    /* end shape 2 */
    /* shape 3 */
    
    Matrix transform_pattern_3_Ka;
    matrix_identity(transform_pattern_3_Ka);
    Matrix transform_pattern_perturbed_3_Ka_0, transform_pattern_perturbed_3_Ka_0_tmp;
    matrix_identity(transform_pattern_perturbed_3_Ka_0);
    matrix_translate(-1.0000000000, 0.0000000000, 0.0000000000, transform_pattern_perturbed_3_Ka_0_tmp);
    transform_chain(transform_pattern_perturbed_3_Ka_0_tmp, transform_pattern_perturbed_3_Ka_0);
    matrix_scale(2.0000000000, 2.0000000000, 2.0000000000, transform_pattern_perturbed_3_Ka_0_tmp);
    transform_chain(transform_pattern_perturbed_3_Ka_0_tmp, transform_pattern_perturbed_3_Ka_0);

    Color pattern_perturbed_3_Ka_0_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_perturbed_3_Ka_0_color_1_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_perturbed_3_Ka_0_color_0;
    Color pattern_perturbed_3_Ka_0_color_1;
    color_space_fn(pattern_perturbed_3_Ka_0_color_0_raw, pattern_perturbed_3_Ka_0_color_0);
    color_space_fn(pattern_perturbed_3_Ka_0_color_1_raw, pattern_perturbed_3_Ka_0_color_1);
    Pattern pattern_perturbed_3_Ka_0 = gradient_pattern_alloc(pattern_perturbed_3_Ka_0_color_0, pattern_perturbed_3_Ka_0_color_1);

    pattern_set_transform(pattern_perturbed_3_Ka_0, transform_pattern_perturbed_3_Ka_0);

    Pattern pattern_3_Ka = perturbed_pattern_alloc(pattern_perturbed_3_Ka_0, 1.0000000000, 0.0100000000, 0.7000000000, 1, 0);
    pattern_set_transform(pattern_3_Ka, transform_pattern_3_Ka);
Matrix transform_pattern_3_Kd;
    matrix_identity(transform_pattern_3_Kd);
    Matrix transform_pattern_perturbed_3_Kd_0, transform_pattern_perturbed_3_Kd_0_tmp;
    matrix_identity(transform_pattern_perturbed_3_Kd_0);
    matrix_translate(-1.0000000000, 0.0000000000, 0.0000000000, transform_pattern_perturbed_3_Kd_0_tmp);
    transform_chain(transform_pattern_perturbed_3_Kd_0_tmp, transform_pattern_perturbed_3_Kd_0);
    matrix_scale(2.0000000000, 2.0000000000, 2.0000000000, transform_pattern_perturbed_3_Kd_0_tmp);
    transform_chain(transform_pattern_perturbed_3_Kd_0_tmp, transform_pattern_perturbed_3_Kd_0);

    Color pattern_perturbed_3_Kd_0_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_perturbed_3_Kd_0_color_1_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_perturbed_3_Kd_0_color_0;
    Color pattern_perturbed_3_Kd_0_color_1;
    color_space_fn(pattern_perturbed_3_Kd_0_color_0_raw, pattern_perturbed_3_Kd_0_color_0);
    color_space_fn(pattern_perturbed_3_Kd_0_color_1_raw, pattern_perturbed_3_Kd_0_color_1);
    Pattern pattern_perturbed_3_Kd_0 = gradient_pattern_alloc(pattern_perturbed_3_Kd_0_color_0, pattern_perturbed_3_Kd_0_color_1);

    pattern_set_transform(pattern_perturbed_3_Kd_0, transform_pattern_perturbed_3_Kd_0);

    Pattern pattern_3_Kd = perturbed_pattern_alloc(pattern_perturbed_3_Kd_0, 1.0000000000, 0.0100000000, 0.7000000000, 1, 0);
    pattern_set_transform(pattern_3_Kd, transform_pattern_3_Kd);
    Pattern pattern_3_Ks = NULL;
    Pattern pattern_3_Ns = NULL;
    Pattern pattern_3_bump = NULL;
    Pattern pattern_3_disp = NULL;
    Pattern pattern_3_refl = NULL;
    Pattern pattern_3_d = NULL;
    Color material_3_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_3_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_3_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_3 = material_alloc();
    color_space_fn(material_3_color_raw, material_3->Ka);
    color_space_fn(material_3_color_raw, material_3->Kd);
    color_space_fn(material_3_color_raw, material_3->Ks);
    color_scale(material_3->Ka, 0.1000000000);
    color_scale(material_3->Kd, 0.7000000000);
    color_scale(material_3->Ks, 0.3000000000);
    rgb_to_rgb(material_3_reflective, material_3->refl);
    rgb_to_rgb(material_3_refractive, material_3->Tf);
    material_3->reflective = material_3_reflective[0] > 0.0
                             || material_3_reflective[1] > 0.0
                             || material_3_reflective[2] > 0.0;

    material_3->Tr = 0.0000000000;
    material_3->Ns = 50.0000000000;
    material_3->Ni = 1.0000000000;
    material_3->casts_shadow = true;
    material_set_pattern(material_3, map_Ka, pattern_3_Ka);
    material_set_pattern(material_3, map_Kd, pattern_3_Kd);
    material_set_pattern(material_3, map_Ks, pattern_3_Ks);
    material_set_pattern(material_3, map_Ns, pattern_3_Ns);
    material_set_pattern(material_3, map_d, pattern_3_d);
    material_set_pattern(material_3, map_bump, pattern_3_bump);
    material_set_pattern(material_3, map_disp, pattern_3_disp);
    material_set_pattern(material_3, map_refl, pattern_3_refl);

    Matrix transform_3;
    matrix_translate(2.2000000000, 1.0000000000, 0.5000000000, transform_3);
    Shape shape_3 = all_shapes + 3;
    sphere(shape_3);
    shape_set_material(shape_3, material_3);
    shape_set_transform(shape_3, transform_3);

    /* end shape 3 */
    /* end shapes */

    Shape world_group = array_of_shapes(1);
    group(world_group, all_shapes, 4);
    printf("Balancing scene...");
    fflush(stdout);
    world_group->divide(world_group, global_config.scene.divide_threshold);
    printf("Done!\n");
    fflush(stdout);

    World w = world();
    w->lights = all_lights;
    w->lights_num = 1;
    w->shapes = world_group;
    w->shapes_num = 1;
    w->global_config = &global_config;

    if (global_config.illumination.gi.photon_count > 0 && (global_config.illumination.include_global  || global_config.illumination.debug_visualize_photon_map || global_config.illumination.debug_visualize_soft_indirect)) {
        w->photon_maps = array_of_photon_maps(3);
        printf("Tracing photons...");
        fflush(stdout);
        int i;
        for (i = 0; i < 3; ++i) {
            init_Photon_map(global_config.illumination.gi.photon_count, w->photon_maps + i);
        }
        trace_photons(w, 3, global_config.illumination.gi.include_caustics, global_config.illumination.gi.include_final_gather);
        printf("Done!\n");
        fflush(stdout);
    } else {
        w->photon_maps = NULL;
        printf("Skipping photon tracing because photon_count is 0.\n");
        fflush(stdout);
    }

    Canvas c = render_multi(cam, w, cam->usteps, cam->vsteps, cam->aperture.jitter);

    write_ppm_file(c, true, global_config.output.file_path);
    write_png(c, global_config.output.file_path);

    canvas_free(c);

    return 0;
}

